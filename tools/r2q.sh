#!/bin/bash
# Historical (r02): the FIELD_FWD_PF variants were removed after this run
# (profiles/r02_field_fwd_prefetch_depth.log).
# Field forward prefetch-depth A/B (FIELD_FWD_PF) on the bench shape, then the field GPU
# tests and one bench run with the product library.
set -o pipefail
mkdir -p gpurun_out/r2q
for v in pf1 pf2 pf2w3 pf4 prod; do
  echo "== $v"
  if [ $v = prod ]; then unset ANR_HIP_LIB; else export ANR_HIP_LIB=$PWD/exp_libs/libanr_ff_$v.so; fi
  timeout -k 10 120 python -u tools/field_probe.py --iters 10 || exit $?
done
unset ANR_HIP_LIB
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "field" > gpurun_out/r2q/tests.log 2>&1 || { tail -30 gpurun_out/r2q/tests.log; exit 1; }
tail -3 gpurun_out/r2q/tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r2q/bench.log 2>&1 || { tail -30 gpurun_out/r2q/bench.log; exit 1; }
tail -1 gpurun_out/r2q/bench.log | cut -c1-400
