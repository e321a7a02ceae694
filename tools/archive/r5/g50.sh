#!/bin/bash
# r5: hash-grid backward variants timed on the settled reference-numerics step's own inputs
# (tools/r5/hash_bwd_state.py), all with the max-ILP scheduler: prefetch batch 6 (the
# default) against 4, 5 and 7
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g50; mkdir -p $O
timeout -k 10 400 python -u tools/r5/hash_bwd_state.py dump --steps 150 --out /tmp/hb_state.pt > $O/dump.log 2>&1 || { tail -20 $O/dump.log; exit 1; }
tail -3 $O/dump.log
for rep in 1 2; do
for v in bs6 bs4 bs5 bs7; do
ANR_HIP_LIB=$PWD/exp_libs/$v.so timeout -k 10 200 python -u tools/r5/hash_bwd_state.py time --state /tmp/hb_state.pt --iters 30 > $O/time_${v}_$rep.log 2>&1 || { tail -20 $O/time_${v}_$rep.log; exit 1; }
echo "$v rep $rep: $(tail -1 $O/time_${v}_$rep.log)"
done
done
