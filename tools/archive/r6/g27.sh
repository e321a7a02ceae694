#!/bin/bash
# r6: hashed levels hash byte-scaled components, the level base as the loads SGPR offset
# (in-tree H1) against the committed library (ab/libanr_H0.so); bit-identity tests first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g27; mkdir -p $O
L=$PWD/atmospheric-neural-rendering_amd/atmonr_amd/_native/ab
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "hashgrid or planes or hash_field" > $O/test_kern.log 2>&1 || { tail -40 $O/test_kern.log; exit 1; }
tail -n 1 $O/test_kern.log
for rep in 1 2 3; do
  for v in H0 H1; do
    if [ $v = H1 ]; then unset ANR_HIP_LIB; else export ANR_HIP_LIB=$L/libanr_$v.so; fi
    timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
    python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "$v $rep"
  done
done
