#!/bin/bash
# r6 final: rocprofv3 kernel trace + FETCH / WRITE / ATOMIC PMC passes (tools/prof.sh) and
# the SQ / TA / TCP counter passes (tools/sq_bench.sh) of the bench step; summaries copied
# to gpurun_out (the raw CSVs are removed: the merge-back limit is 64 MiB)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06_final}
O=gpurun_out/$T; mkdir -p $O
bash tools/prof.sh $O/prof > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/prof_summary.py $O/prof $T > $O/summary_print.log 2>&1 || { tail -20 $O/summary_print.log; exit 1; }
cp profiles/${T}_summary.md profiles/${T}_kernel_stats.csv profiles/pmc_traffic.json $O/
bash tools/sq_bench.sh $O/sq > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
python3 tools/pmc_table.py $O/sq > $O/sq_table.txt
rm -rf $O/prof $O/sq
echo done
