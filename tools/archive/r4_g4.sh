set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ref16_gpu.py tests/test_kernels_gpu.py -k "ref16 or hashgrid" > gpurun_out/r4_ref16_test.log 2>&1 || { tail -40 gpurun_out/r4_ref16_test.log; exit 1; }
tail -3 gpurun_out/r4_ref16_test.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --numerics reference > gpurun_out/r4_bench_ref.json.log 2>&1 && tail -c 600 gpurun_out/r4_bench_ref.json.log
timeout -k 10 300 python -u bench.py --batch 1024 --graph on --no-cpu-baseline --no-alt-numerics > gpurun_out/r4_b1024_graph.json.log 2>&1; tail -c 600 gpurun_out/r4_b1024_graph.json.log
