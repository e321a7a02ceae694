set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_graph_gpu.py tests/test_extract_gpu.py > gpurun_out/r4_graph_test.log 2>&1 || { tail -60 gpurun_out/r4_graph_test.log; exit 1; }
tail -5 gpurun_out/r4_graph_test.log
timeout -k 10 300 python -u bench.py --batch 1024 --graph off --no-cpu-baseline --no-alt-numerics > gpurun_out/r4_b1024_eager.json.log 2>&1 && tail -c 600 gpurun_out/r4_b1024_eager.json.log &&
timeout -k 10 300 python -u bench.py --batch 1024 --graph on --no-cpu-baseline --no-alt-numerics > gpurun_out/r4_b1024_graph.json.log 2>&1 && tail -c 1500 gpurun_out/r4_b1024_graph.json.log &&
timeout -k 10 300 python -u bench.py --workload extract --steps 20 --cpu-budget 15 > gpurun_out/r4_extract.json.log 2>&1 && tail -c 2500 gpurun_out/r4_extract.json.log &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r4_bench.json.log 2>&1 && tail -c 3000 gpurun_out/r4_bench.json.log
