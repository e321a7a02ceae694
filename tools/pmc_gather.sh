#!/bin/bash
# FETCH_SIZE and TCC hit/miss of the 4-B gather calibration kernel (known byte counts,
# tools/ubench/gather_calib.py) and of the bench step's kernels, in separate PMC passes.
set -o pipefail
OUT=${1:-gpurun_out/pmc_gather}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/ubench/gather_calib.py --out "$OUT/gather_times.json" > "$OUT/times.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/ub_fetch" -o run --output-format csv -- python3 tools/ubench/gather_calib.py > "$OUT/ub_fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/ub_hit" -o run --output-format csv -- python3 tools/ubench/gather_calib.py > "$OUT/ub_hit.log" 2>&1 || exit $?
ARGS="--steps 3 --warmup 12 --no-cpu-baseline --no-kernel-timer --spec-peaks"
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/bench_hit" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_hit.log" 2>&1 || exit $?
echo done
