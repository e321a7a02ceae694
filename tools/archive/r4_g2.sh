set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --batch 1024 --graph on --no-cpu-baseline --no-alt-numerics > gpurun_out/r4_b1024_graph.json.log 2>&1; tail -c 2500 gpurun_out/r4_b1024_graph.json.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r4_bench.json.log 2>&1 && tail -c 1200 gpurun_out/r4_bench.json.log && bash tools/r4_g3.sh
