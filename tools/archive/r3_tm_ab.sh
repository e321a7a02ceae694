#!/bin/bash
# Same-box A/B of the composite -> field per-tile maxima hand-off (ANR_TILE_MAX=1, default)
# against the two-pass form (0: the field's own absmax kernel), alternating, 20 timed steps.
set -o pipefail
OUT=${1:-gpurun_out/tm_ab}; mkdir -p "$OUT"
for i in 1 2 3; do
  for v in 0 1; do
    ANR_TILE_MAX=$v timeout -k 10 300 python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline \
      > "$OUT/bench_tm${v}_$i.log" 2>&1 || exit $?
  done
done
echo done
