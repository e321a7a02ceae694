# Alternating A/B bench pairs of an environment variable (same library, one box):
#   VAR=ANR_HASH_SKIP0 VALS="1 2" REPS=2 TAG=x BENCH_ARGS=... bash tools/r5/ab_env.sh
# Optional TESTS="tests/test_kernels_gpu.py -k hash" run first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ab}
mkdir -p gpurun_out/$TAG
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > gpurun_out/$TAG/test.log 2>&1 || { tail -40 gpurun_out/$TAG/test.log; exit 1; }
  tail -1 gpurun_out/$TAG/test.log
fi
for rep in $(seq 1 ${REPS:-2}); do
for v in $VALS; do
env $VAR=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-numerics ${BENCH_ARGS} > gpurun_out/$TAG/${v}_$rep.json.log 2>&1 || { tail -20 gpurun_out/$TAG/${v}_$rep.json.log; exit 1; }
python3 tools/r5/bench_line.py gpurun_out/$TAG/${v}_$rep.json.log "$VAR=$v rep $rep"
done
done
