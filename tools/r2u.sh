#!/bin/bash
# Historical (r02): the FIELD_BWD_KEEP experiment macro became the product code after
# this run (profiles/r02_field_bwd_keep.log).
# Field backward: keep the previous tile's raw directions (KEEP=1) and d_sigma (KEEP=2)
# live to the end of the iteration, so the loop-carried copies of the prefetched inputs
# move to the iteration's end (no mid-tile vmcnt wait). Probe A/B vs the product library,
# then the field GPU tests with the better variant.
set -o pipefail
for v in prod keep keep2 prod keep keep2; do
  echo "== $v"
  if [ $v = prod ]; then unset ANR_HIP_LIB; else export ANR_HIP_LIB=$PWD/exp_libs/libanr_ff_$v.so; fi
  timeout -k 10 120 python -u tools/field_probe.py --iters 10 || exit $?
done
export ANR_HIP_LIB=$PWD/exp_libs/libanr_ff_keep2.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "field" 2>&1 | tail -2
