#!/bin/bash
# Field backward ablations (FIELD_EXP bits, see field_fused.hip) and per-stage s_memtime
# stamps on the bench shape (tools/field_probe.py), from libraries built into build_exp/.
set -o pipefail
for v in base stamp exp1 exp2 exp4 exp8 exp15; do
  echo "== $v"
  if [ $v = base ]; then lib=""; else lib="ANR_HIP_LIB=$PWD/build_exp/libanr_ff_$v.so"; fi
  env $lib timeout -k 10 120 python -u tools/field_probe.py --iters 5 || exit $?
done
