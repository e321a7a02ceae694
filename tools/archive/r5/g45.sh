#!/bin/bash
# r5: reference numerics' dL/denc as f16 between the field and hash-grid backwards
# (ANR_DENC_F16=1) vs f32 (0): kernel + pipeline tests, then alternating bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g45; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_ref16_gpu.py tests/test_pipeline_gpu.py -k "ref16 or field or hashgrid or pipeline" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2 3; do
for v in 1 0; do
ANR_DENC_F16=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-numerics > $O/h${v}_$rep.json.log 2>&1 || { tail -20 $O/h${v}_$rep.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/h${v}_$rep.json.log "denc_f16=$v rep $rep"
done
done
