#!/bin/bash
# r03: bench.py A/B of two environments on one box, alternating, one JSON line each.
# usage: tools/r3_bench_ab.sh <out-dir> "<env A>" "<env B>" [pytest -k expr]
set -o pipefail
OUT=$1; A=$2; B=$3; K=$4; mkdir -p "$OUT"
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -k "$K" -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
for r in 1 2; do
  for tag in A B; do
    if [ $tag = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench_${tag}$r.json.log" 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_ms'])" "$OUT/bench_${tag}$r.json.log" "$tag$r [$E]"
  done
done
