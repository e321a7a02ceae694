#!/bin/bash
# r6: SQ / TA / TCP counters of the fused hash-grid + field forward against the two-kernel
# forward, same box (tools/sq_bench.sh passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g8; mkdir -p $O
bash tools/sq_bench.sh $O/fused > $O/fused.log 2>&1 || { tail -20 $O/fused.log; exit 1; }
ANR_HASH_FIELD=0 bash tools/sq_bench.sh $O/two > $O/two.log 2>&1 || { tail -20 $O/two.log; exit 1; }
python3 tools/pmc_table.py $O/fused > $O/fused_table.txt
python3 tools/pmc_table.py $O/two > $O/two_table.txt
rm -rf $O/fused $O/two
