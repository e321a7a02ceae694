#!/bin/bash
# Memory-side atomic request counts (TCC_EA0_ATOMIC_sum, 64-B requests) for the ubench
# calibration kernels (known request counts) and for the bench step's kernels.
set -o pipefail
OUT=gpurun_out/${1:-pmc_atomic}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 12 --no-cpu-baseline --no-kernel-timer --spec-peaks ${BENCH_ARGS}"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d "$OUT/ub" -o run --output-format csv -- python3 tools/ubench/peaks.py > "$OUT/ub.log" 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d "$OUT/bench" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/bench.log" 2>&1 || exit $?
echo done
