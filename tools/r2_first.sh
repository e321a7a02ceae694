#!/bin/bash
# Round-2 first GPU pass: measured peaks, the default bench, the --gpus 2 launcher
# (gloo, both ranks on the box's one GPU), gpu tests, counter list.
set -o pipefail
OUT=gpurun_out/${1:-r2a}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/ubench/peaks.py > "$OUT/peaks.json" 2> "$OUT/peaks.err" || exit $?
timeout -k 10 300 python -u bench.py > "$OUT/bench.log" 2>&1 || exit $?
ANR_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 \
  --no-cpu-baseline > "$OUT/bench_g2_gloo.log" 2>&1 || exit $?
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit $?
echo done
