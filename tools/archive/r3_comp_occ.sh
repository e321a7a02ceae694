#!/bin/bash
# r03: composite backward (rb::bwd_kernel) capped at 6 waves per SIMD (86 -> 80 VGPRs, one
# spill; exp_libs/libanr_cpw6.so) against the product library (5 waves): composite GPU
# tests on the variant, then alternating bench.py runs (ms/step, anr_composite_bwd avg).
# (Record: not kept; profiles/r03_comp_occ.log.)
set -o pipefail
OUT=${1:-gpurun_out/cpw}; mkdir -p "$OUT"
LIB=$PWD/exp_libs/libanr_cpw6.so
ANR_HIP_LIB=$LIB timeout -k 10 400 python -u -m pytest tests -m gpu -k "composite or render" -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2; do
  for v in cand cpw6; do
    if [ $v = cand ]; then lib=""; else lib=$LIB; fi
    env ${lib:+ANR_HIP_LIB=$lib} timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench_$v$r.json.log" 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print(sys.argv[2], d['value'], d['ms_per_step'], 'comp_bwd', k['anr_composite_bwd']['avg_ms'], 'comp_fwd', k['anr_composite_fwd']['avg_ms'])" "$OUT/bench_$v$r.json.log" "$v$r"
  done
done
