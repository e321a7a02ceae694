#!/bin/bash
# r6: fused hash-grid + field forward -- bit-identity tests, step tests, then bench A/B
# (two-kernel forward vs fused at register caps 4 / 5 / 6 waves per SIMD)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g7; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "hash_field_fwd or quad_planes or hashgrid" > $O/test_kern.log 2>&1 || { tail -30 $O/test_kern.log; exit 1; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "train_step or field" tests/test_graph_gpu.py > $O/test_step.log 2>&1 || { tail -30 $O/test_step.log; exit 1; }
for v in two occ6 occ4 occ5 two2 occ6b; do
  case $v in two*) E="ANR_HASH_FIELD=0";; occ6*) E="ANR_HF_OCC=6";; occ4) E="ANR_HF_OCC=4";; occ5) E="ANR_HF_OCC=5";; esac
  env $E timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_$v.json.log 2>&1 || { tail -30 $O/bench_$v.json.log; exit 1; }
  python3 tools/r5/bench_line.py $O/bench_$v.json.log $v
done
