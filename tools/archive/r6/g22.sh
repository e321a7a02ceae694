#!/bin/bash
# r6: X = the committed pos/list-pass library (_native/ab/libanr_X.so); Y = + clear rows
# not written, pos pass capped at 3 waves/SIMD (spills; ab/libanr_Y.so); Z = + clear rows
# not written, pos pass at 2 waves/SIMD (the in-tree library). Kernel tests on Z first.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g22; mkdir -p $O
L=$PWD/atmospheric-neural-rendering_amd/atmonr_amd/_native/ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "rows or zero_color or zero_gradient or bench_size or ingp_field or relaunch or bwd_tiles" > $O/test_kern.log 2>&1 || { tail -40 $O/test_kern.log; exit 1; }
tail -n 1 $O/test_kern.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "train_step or grad or fixed_iterations" tests/test_graph_gpu.py tests/test_pipeline_gpu.py tests/test_liveness_gpu.py > $O/test_step.log 2>&1 || { tail -30 $O/test_step.log; exit 1; }
tail -n 1 $O/test_step.log
for rep in 1 2; do
  for v in X Y Z; do
    if [ $v = Z ]; then unset ANR_HIP_LIB; else export ANR_HIP_LIB=$L/libanr_$v.so; fi
    timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
    python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "$v $rep"
  done
done
