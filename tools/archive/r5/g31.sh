#!/bin/bash
# r5: NeRF dense-layer kernels with uniform load paths + scalar wave index (exp_libs/nerfwait.so)
# against the previous library (exp_libs/base.so): NeRF kernel tests on the new library, the
# GEMM probe and the NeRF bench line on both
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g31; mkdir -p $O
ANR_HIP_LIB=$PWD/exp_libs/nerfwait.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nerf_gpu.py > $O/test_nerf.log 2>&1 || { tail -40 $O/test_nerf.log; exit 1; }
tail -1 $O/test_nerf.log
for v in nerfwait base; do
ANR_HIP_LIB=$PWD/exp_libs/$v.so timeout -k 10 300 python -u tools/r5/nerf_gemm_probe.py > $O/probe_$v.log 2>&1 || { tail -20 $O/probe_$v.log; exit 1; }
echo "== probe $v"; cat $O/probe_$v.log
done
for v in nerfwait base; do
ANR_HIP_LIB=$PWD/exp_libs/$v.so timeout -k 10 300 python -u bench.py --workload nerf --no-cpu-baseline > $O/bench_nerf_$v.json.log 2>&1 || { tail -30 $O/bench_nerf_$v.json.log; exit 1; }
echo "== bench $v"; tail -1 $O/bench_nerf_$v.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline'].get('frac'), d['roofline'].get('gemm_kernels'))"
done
