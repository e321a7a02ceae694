#!/bin/bash
# r6: half-wave x-pair gathers in the hash-grid forward (HASH_XSWAP): bit-identity tests,
# then alternating bench A/B against the HASH_XSWAP=0 build (exp_libs/noxswap), fused forward
# and two-kernel forward
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g10; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "hash_field_fwd or quad_planes or hashgrid" > $O/test_kern.log 2>&1 || { tail -30 $O/test_kern.log; exit 1; }
tail -n 1 $O/test_kern.log
for rep in 1 2; do
for v in xs noxs xs_two noxs_two; do
  E="ANR_X=0"
  case $v in noxs*) E="ANR_HIP_LIB=$GRAFT_REPO_ROOT/exp_libs/noxswap/libanr_hip.so";; esac
  F="ANR_Y=0"; case $v in *_two) F="ANR_HASH_FIELD=0";; esac
  env $E $F timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
  python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "$v $rep"
done
done
