#!/bin/bash
# r03 final: bf16 profile passes, then the whole GPU suite (one process, thread timeouts).
set -o pipefail
OUT=${1:-gpurun_out/final}; mkdir -p "$OUT"
tools/r3_final_prof.sh "$OUT" bf16 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; exit $rc
