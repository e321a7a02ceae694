#!/bin/bash
# r5 final (max-ILP field kernels): rocprof kernel trace + PMC traffic passes over the settled bench step on the final
# library (field-bwd store deferral, NeRF uniform loads)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g44; mkdir -p $O
BENCH_ARGS=--no-alt-numerics STEPS=5 bash tools/prof.sh $O/prof > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
ls $O/prof
