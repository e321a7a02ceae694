#!/bin/bash
# r6: A = first row-bit library (_native/ab/libanr_A.so); B1 = + hash-grid backward walk
# without short-circuit branches and batched LDS row indices (ab/libanr_B1.so); B2 = B1 +
# the reference-numerics field backward skipping the dir network on zero-colour tiles (the
# in-tree library). Kernel tests on B2, then alternating bench runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g20; mkdir -p $O
L=$PWD/atmospheric-neural-rendering_amd/atmonr_amd/_native/ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "rows_equals or bwd_tiles or zero_gradient or zero_color or bench_size or hashgrid_fwd_bwd or request_count or ingp_field or relaunch" > $O/test_kern.log 2>&1 || { tail -40 $O/test_kern.log; exit 1; }
tail -n 1 $O/test_kern.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "train_step or grad or fixed_iterations" tests/test_graph_gpu.py tests/test_pipeline_gpu.py > $O/test_step.log 2>&1 || { tail -30 $O/test_step.log; exit 1; }
tail -n 1 $O/test_step.log
for rep in 1 2; do
  for v in A B1 B2; do
    if [ $v = B2 ]; then unset ANR_HIP_LIB; else export ANR_HIP_LIB=$L/libanr_$v.so; fi
    timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
    python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "$v $rep"
  done
done
