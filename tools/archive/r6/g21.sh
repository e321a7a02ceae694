#!/bin/bash
# r6: reference-numerics field backward as a pos pass (2 waves/SIMD) + a list pass
# (ANR_POS_PASS=1, default) against the one-kernel form (ANR_POS_PASS=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g21; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "rows_equals or zero_color or zero_gradient or bench_size or ingp_field or relaunch" > $O/test_kern.log 2>&1 || { tail -40 $O/test_kern.log; exit 1; }
tail -n 1 $O/test_kern.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "train_step or grad or fixed_iterations" tests/test_graph_gpu.py tests/test_pipeline_gpu.py tests/test_liveness_gpu.py > $O/test_step.log 2>&1 || { tail -30 $O/test_step.log; exit 1; }
tail -n 1 $O/test_step.log
for rep in 1 2 3; do
  for v in 0 1; do
    ANR_POS_PASS=$v timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
    python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "pospass $v $rep"
  done
done
