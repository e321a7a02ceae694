#!/bin/bash
# r6: reference-numerics dL/denc as f16 rows + per-row bits, hash-grid backward walks only
# the set rows (ANR_ROW_BITS, default 1) -- kernel tests, step tests, then alternating A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g18; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "rows_equals or bwd_tiles or zero_gradient or relaunch or bench_size_adjoint" > $O/test_kern.log 2>&1 || { tail -40 $O/test_kern.log; exit 1; }
tail -n 1 $O/test_kern.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "train_step or deferred or grad" tests/test_graph_gpu.py tests/test_pipeline_gpu.py > $O/test_step.log 2>&1 || { tail -30 $O/test_step.log; exit 1; }
tail -n 1 $O/test_step.log
for rep in 1 2 3; do
for v in 0 1; do
  ANR_ROW_BITS=$v timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
  python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "rowbits $v $rep"
done
done
