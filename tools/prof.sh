#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate PMC passes (TCC slots: they do not fit together on gfx950), then
# TCC_EA0_ATOMIC_sum (memory-side atomic requests). Steady state: 12 warm-up steps.
set -o pipefail
OUT=${1:-gpurun_out/prof}
STEPS=${STEPS:-5}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps $STEPS --warmup 12 --no-cpu-baseline --no-kernel-timer --spec-peaks ${BENCH_ARGS}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1 || exit $?
timeout -s KILL 600 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d "$OUT/atomic" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/atomic.log" 2>&1 || exit $?
echo done
