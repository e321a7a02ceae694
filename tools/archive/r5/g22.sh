#!/bin/bash
# r5: hash-grid backward samples-per-wave (K) A/B under the reference numerics
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_g22; mkdir -p $O
for k in 64 128 192 256; do
ANR_HASH_KB=$k timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/ref_k$k.json.log 2>&1 || { tail -30 $O/ref_k$k.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/ref_k$k.json.log ref_k$k
done
