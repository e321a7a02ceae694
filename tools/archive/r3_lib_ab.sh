#!/bin/bash
# r03: same-box A/B of the product library against a saved baseline library
# (exp_libs/libanr_base.so) on one profiling tool; optional pytest -k filter first.
# usage: tools/r3_lib_ab.sh <out-dir> "<pytest -k expr or ''>" <tool.py args...>
set -o pipefail
OUT=$1; K=$2; shift 2; mkdir -p "$OUT"
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -k "$K" -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
for r in 1 2; do
  echo "== base ($r)"; ANR_HIP_LIB=$PWD/exp_libs/libanr_base.so timeout -k 10 300 python -u "$@" 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== cand ($r)"; timeout -k 10 300 python -u "$@" 2>&1 | grep -v amdgpu.ids || exit 1
done
