#!/bin/bash
# r6: list pass with a block-uniform early exit when the list has no tile for the block
# (L1, in-tree) against the committed library (L0, ab/libanr_L0.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g32; mkdir -p $O
L=$PWD/atmospheric-neural-rendering_amd/atmonr_amd/_native/ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "rows or zero_color" tests/test_graph_gpu.py tests/test_ingp_oracle_gpu.py -k "rows or zero_color or train_step or graph or adam" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -n 1 $O/test.log
for rep in 1 2 3; do
  for v in L0 L1; do
    if [ $v = L1 ]; then unset ANR_HIP_LIB; else export ANR_HIP_LIB=$L/libanr_$v.so; fi
    timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
    python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "$v $rep"
  done
done
