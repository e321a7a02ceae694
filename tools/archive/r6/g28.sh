#!/bin/bash
# r6: planes forward: lane constants once per quad, follower values left undefined, DPP with
# bound_ctrl (no per-corner or per-dimension fills)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g28; mkdir -p $O
L=$PWD/atmospheric-neural-rendering_amd/atmonr_amd/_native/ab
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "hashgrid or planes or hash_field" > $O/test_kern.log 2>&1 || { tail -40 $O/test_kern.log; exit 1; }
tail -n 1 $O/test_kern.log
for rep in 1 2 3; do
  for v in K0 K1; do
    if [ $v = K1 ]; then unset ANR_HIP_LIB; else export ANR_HIP_LIB=$L/libanr_$v.so; fi
    timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/bench_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_${v}_$rep.json.log; exit 1; }
    python3 tools/r5/bench_line.py $O/bench_${v}_$rep.json.log "$v $rep"
  done
done
