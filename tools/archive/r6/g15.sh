#!/bin/bash
# r6: field forward with LDS weight fragments (ANR_FIELD_FWD_LDS 6 / 8) -- the field tests
# under it (the uniform-tile form against the general form, bit for bit), then alternating
# bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g15; mkdir -p $O
ANR_FIELD_FWD_LDS=8 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "field" > $O/test8.log 2>&1 || { tail -30 $O/test8.log; exit 1; }
tail -n 1 $O/test8.log
ANR_FIELD_FWD_LDS=6 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "field" > $O/test6.log 2>&1 || { tail -30 $O/test6.log; exit 1; }
tail -n 1 $O/test6.log
for rep in 1 2; do
for v in 0 6 8; do
  ANR_FIELD_FWD_LDS=$v timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
  python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "fwd_lds $v $rep"
done
done
