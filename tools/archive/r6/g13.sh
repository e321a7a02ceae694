#!/bin/bash
# r6: run-leader threshold of the hash-grid forward (ANR_HASH_DEDUP 16 / 32 / 48 / 64 / 0),
# two-kernel forward, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g13; mkdir -p $O
for rep in 1 2; do
for v in 32 16 48 64 0; do
  ANR_HASH_DEDUP=$v timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
  python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "dedup $v $rep"
done
done
