#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench, rocprofv3 kernel trace of a short bench.
# Usage (via gpurun): bash tools/gpu_check.sh [tag]   -> gpurun_out/<tag>/*
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  ANR_PSNR_OUT=$OUT/psnr.json ANR_INGP_PSNR_OUT=$OUT/psnr_ingp.json timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit $?
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > "$OUT/bench.log" 2>&1 || exit $?
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timer ${BENCH_ARGS} > "$OUT/trace.log" 2>&1 || exit $?
fi
echo done
