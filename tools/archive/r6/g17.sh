#!/bin/bash
# r6: split backward (ANR_BWD_SPLIT=1: first half's hash-grid backward on an auxiliary
# stream beside the second half's field backward) -- step tests under it, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g17; mkdir -p $O
ANR_BWD_SPLIT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "train_step or deferred or grad" tests/test_graph_gpu.py tests/test_pipeline_gpu.py > $O/test_split.log 2>&1 || { tail -30 $O/test_split.log; exit 1; }
tail -n 1 $O/test_split.log
for rep in 1 2 3; do
for v in 0 1; do
  ANR_BWD_SPLIT=$v timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
  python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "split $v $rep"
done
done
