#!/bin/bash
# r6: hash-grid dense-level wrap without per-corner branches (hash_levels.h dense_wrap) in
# the planes forward and the backward walkers; row walker chunks rounded to 32-row words.
# X = the committed library (_native/ab/libanr_X.so), N = the in-tree library.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g23; mkdir -p $O
L=$PWD/atmospheric-neural-rendering_amd/atmonr_amd/_native/ab
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "hashgrid or rows or planes or hash_field or zero_color" > $O/test_kern.log 2>&1 || { tail -40 $O/test_kern.log; exit 1; }
tail -n 1 $O/test_kern.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "train_step or grad or fixed_iterations" tests/test_graph_gpu.py tests/test_pipeline_gpu.py > $O/test_step.log 2>&1 || { tail -30 $O/test_step.log; exit 1; }
tail -n 1 $O/test_step.log
for rep in 1 2 3; do
  for v in X N; do
    if [ $v = N ]; then unset ANR_HIP_LIB; else export ANR_HIP_LIB=$L/libanr_$v.so; fi
    timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
    python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "$v $rep"
  done
done
