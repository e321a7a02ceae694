#!/bin/bash
# Hash-grid kernel variants on the bench geometry (tools/hash_probe.py), one line each.
set -o pipefail
run() {  # label, env...
  local label=$1; shift
  echo "== $label"
  env "$@" timeout -k 10 120 python -u tools/hash_probe.py --iters 5 || exit $?
}
run "v1 lpw16"        ANR_HASHGRID_MODE=3
run "v1 lpw2"         ANR_HASHGRID_MODE=3 ANR_HASH_LPW=2
run "v3 bs8 lpw16"    ANR_HASHGRID_MODE=0
run "v3 bs8 lpw4"     ANR_HASHGRID_MODE=0 ANR_HASH_LPW=4
run "v3 bs8 lpw2"     ANR_HASHGRID_MODE=0 ANR_HASH_LPW=2
run "v3 bs4 lpw16"    ANR_HASHGRID_MODE=0 ANR_HIP_LIB=$PWD/build_exp/libanr_bs4.so
run "v3 bs4 lpw2"     ANR_HASHGRID_MODE=0 ANR_HASH_LPW=2 ANR_HIP_LIB=$PWD/build_exp/libanr_bs4.so
run "v3 bs16 lpw16"   ANR_HASHGRID_MODE=0 ANR_HIP_LIB=$PWD/build_exp/libanr_bs16.so
