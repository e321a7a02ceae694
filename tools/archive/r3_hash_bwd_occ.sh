#!/bin/bash
# r03: hash backward occupancy sweep (prefetch batch HASH_BS x waves-per-SIMD cap) with and
# without x-carry (modes 0 / 8): exp_libs/libanr_<variant>.so against the product library.
# (Record: the exp_libs variants were built from hashgrid.hip with -DHASH_BS / amdgpu_waves_per_eu on the x-carry kernel, removed after the run.)
set -o pipefail
OUT=${1:-gpurun_out/occ}; mkdir -p "$OUT"
for r in 1 2; do
  for v in cand bs6 bs4 bs4w8; do
    if [ $v = cand ]; then lib=""; else lib="$PWD/exp_libs/libanr_$v.so"; fi
    echo "== $v ($r)"
    env ${lib:+ANR_HIP_LIB=$lib} timeout -k 10 200 python -u tools/hash_bwd_ab.py --modes 0,8 --iters 30 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
