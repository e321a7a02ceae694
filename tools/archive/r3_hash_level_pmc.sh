#!/bin/bash
# Per-level hash-forward anatomy (tools/hash_level_probe.py): HIP-event times, then
# TCC hit/miss and FETCH_SIZE / WRITE_SIZE in separate rocprofv3 --pmc passes.
set -o pipefail
OUT=${1:-gpurun_out/hash_levels}
mkdir -p "$OUT"
export TMPDIR=/tmp
P="tools/hash_level_probe.py --reps 3"
timeout -k 10 180 python3 $P --out "$OUT/levels.json" > "$OUT/times.log" 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/hit" -o run --output-format csv -- python3 $P > "$OUT/hit.log" 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 $P > "$OUT/fetch.log" 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 $P > "$OUT/write.log" 2>&1 || exit $?
echo done
