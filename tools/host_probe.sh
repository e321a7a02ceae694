#!/bin/bash
# Host-issue vs GPU time per step: default bench, without the live kernel timer, and long.
set -o pipefail
OUT=${1:-gpurun_out/host}
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/b_default.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-kernel-timer --steps 100 > "$OUT/b_nt100.log" 2>&1 || exit $?
echo done
