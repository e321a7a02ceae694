#!/bin/bash
# Kernel traces of the bench step with and without the per-tile maxima hand-off.
set -o pipefail
OUT=${1:-gpurun_out/tm_trace}; mkdir -p "$OUT"; export TMPDIR=/tmp
ARGS="--steps 5 --warmup 12 --no-cpu-baseline --no-kernel-timer --spec-peaks"
for v in 0 1; do
  ANR_TILE_MAX=$v timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tm$v" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/tm$v.log" 2>&1 || exit $?
done
echo done
