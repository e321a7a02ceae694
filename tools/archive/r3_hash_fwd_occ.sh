#!/bin/bash
# r03: hash forward (v6) coordinate-prefetch depth HASH_FBS x occupancy sweep:
# exp_libs/libanr_<variant>.so against the product library (FBS 4, 88 VGPRs, 5 waves/SIMD).
# (Record: the exp_libs variants were built from hashgrid.hip with -DHASH_FBS / amdgpu_waves_per_eu(6); none kept.)
set -o pipefail
for r in 1 2; do
  for v in cand fbs1 fbs2 fbs3w6; do
    if [ $v = cand ]; then lib=""; else lib="$PWD/exp_libs/libanr_$v.so"; fi
    echo "== $v ($r)"
    env ${lib:+ANR_HIP_LIB=$lib} timeout -k 10 200 python -u tools/hash_fwd_ab.py --modes 0 --iters 30 --views 90 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
