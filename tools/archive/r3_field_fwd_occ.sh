#!/bin/bash
# r03: field forward at 4 waves per SIMD (amdgpu_waves_per_eu(4): 136 -> 126 VGPRs,
# exp_libs/libanr_ffw4.so) against the product library (3 waves): field GPU tests on the
# variant, then alternating bench.py runs (ms/step, profiling-pass field_fwd avg).
# (Record: the variant is now the product form, field_fused.hip fwd_kernel.)
set -o pipefail
OUT=${1:-gpurun_out/ffw}; mkdir -p "$OUT"
LIB=$PWD/exp_libs/libanr_ffw4.so
ANR_HIP_LIB=$LIB timeout -k 10 400 python -u -m pytest tests -m gpu -k "field or ingp" -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2; do
  for v in cand ffw4; do
    if [ $v = cand ]; then lib=""; else lib=$LIB; fi
    env ${lib:+ANR_HIP_LIB=$lib} timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench_$v$r.json.log" 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print(sys.argv[2], d['value'], d['ms_per_step'], 'field_fwd', k['field_fwd']['avg_ms'], 'field_bwd', k['field_bwd']['avg_ms'])" "$OUT/bench_$v$r.json.log" "$v$r"
  done
done
