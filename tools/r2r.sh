#!/bin/bash
# Historical (r02): the libanr_ff_{nm2,ld1,ld1nm2} variants were built from experiment
# macros that were removed after this run (profiles/r02_field_fwd_prefetch_depth.log).
# Field forward A/B: two 16-sample tiles per step (FIELD_FWD_NM=2) and the dir hidden
# layer's weights in LDS (FIELD_FWD_LDS_D1=1: 118 VGPRs, 4 waves/SIMD), tools/field_probe.py.
set -o pipefail
for v in prod nm2 ld1 ld1nm2 prod; do
  echo "== $v"
  if [ $v = prod ]; then unset ANR_HIP_LIB; else export ANR_HIP_LIB=$PWD/exp_libs/libanr_ff_$v.so; fi
  timeout -k 10 120 python -u tools/field_probe.py --iters 10 || exit $?
done
