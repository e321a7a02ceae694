#!/bin/bash
# r5: every other kernel file also built with -mllvm -amdgpu-sched-strategy=max-ilp
# (exp_libs/allilp.so) against the library with it on field_fused only (exp_libs/cur.so):
# kernel / NeRF / ref16 tests on allilp, then alternating INGP and NeRF bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g42; mkdir -p $O
ANR_HIP_LIB=$PWD/exp_libs/allilp.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_nerf_gpu.py tests/test_ref16_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2; do
for v in allilp cur; do
ANR_HIP_LIB=$PWD/exp_libs/$v.so timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-numerics > $O/${v}_$rep.json.log 2>&1 || { tail -20 $O/${v}_$rep.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/${v}_$rep.json.log "$v rep $rep"
done
done
for v in allilp cur; do
ANR_HIP_LIB=$PWD/exp_libs/$v.so timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-numerics --numerics build > $O/${v}_build.json.log 2>&1 || { tail -20 $O/${v}_build.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/${v}_build.json.log "$v build"
done
for v in allilp cur; do
ANR_HIP_LIB=$PWD/exp_libs/$v.so timeout -k 10 300 python -u bench.py --workload nerf --no-cpu-baseline > $O/nerf_$v.json.log 2>&1 || { tail -30 $O/nerf_$v.json.log; exit 1; }
echo "nerf $v: $(tail -1 $O/nerf_$v.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline'].get('gemm_kernels', {}).get('ms_per_step'))")"
done
