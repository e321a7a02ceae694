#!/bin/bash
# r5: SQ counter passes over the settled bench step (tools/sq_bench.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g13; mkdir -p $O
BENCH_ARGS=--no-alt-numerics bash tools/sq_bench.sh $O/sq > $O/sq.log 2>&1 || { tail -30 $O/sq.log; exit 1; }
python3 tools/pmc_table.py $O/sq > $O/sq_table.txt
cat $O/sq_table.txt | head -80
