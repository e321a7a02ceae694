#!/bin/bash
# r5: SQ counter passes over the settled bench step after the field-backward store deferral
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g30; mkdir -p $O
BENCH_ARGS=--no-alt-numerics bash tools/sq_bench.sh $O/sq > $O/sq.log 2>&1 || { tail -30 $O/sq.log; exit 1; }
python3 tools/pmc_table.py $O/sq > $O/sq_table.txt
rm -rf $O/sq/p1 $O/sq/p2 $O/sq/p3
awk '/== field_bwd/,/^== [^f]/' $O/sq_table.txt
