#!/bin/bash
# r6: per-rank strong-scaling shape (1,024 rays x 1,024 samples, hipGraph replay):
# hash-grid backward chunk length (ANR_HASH_KB 64 / 128 / 256) in reference numerics
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g16; mkdir -p $O
for rep in 1 2; do
for k in 256 128 64; do
  ANR_HASH_KB=$k timeout -k 10 300 python -u bench.py --batch 1024 --no-alt-numerics --no-cpu-baseline > $O/b1024_k${k}_$rep.json.log 2>&1 || { tail -30 $O/b1024_k${k}_$rep.json.log; exit 1; }
  python3 tools/r5/bench_line.py $O/b1024_k${k}_$rep.json.log "b1024 K=$k $rep"
done
done
