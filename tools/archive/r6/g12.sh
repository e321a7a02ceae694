#!/bin/bash
# r6: forward variants, alternating, one box: two-kernel forward with / without run-leader
# gathers (ANR_HASH_DEDUP), fused forward without / with them at register caps 4-6
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g12; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "hash_field_fwd or quad_planes or hashgrid" > $O/test_kern.log 2>&1 || { tail -30 $O/test_kern.log; exit 1; }
tail -n 1 $O/test_kern.log
ANR_HF_DEDUP=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "hash_field_fwd" > $O/test_hfdd.log 2>&1 || { tail -30 $O/test_hfdd.log; exit 1; }
tail -n 1 $O/test_hfdd.log
for rep in 1 2; do
for v in two_dd two_nodd hf6 hf6dd hf5dd hf4dd; do
  case $v in
    two_dd) E="ANR_HASH_FIELD=0 ANR_HASH_DEDUP=1";;
    two_nodd) E="ANR_HASH_FIELD=0 ANR_HASH_DEDUP=0";;
    hf6) E="ANR_HF_OCC=6 ANR_HF_DEDUP=0";;
    hf6dd) E="ANR_HF_OCC=6 ANR_HF_DEDUP=1";;
    hf5dd) E="ANR_HF_OCC=5 ANR_HF_DEDUP=1";;
    hf4dd) E="ANR_HF_OCC=4 ANR_HF_DEDUP=1";;
  esac
  env $E timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
  python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "$v $rep"
done
done
