#!/bin/bash
# r5: field_fused.hip compiled with -mllvm -amdgpu-sched-strategy=max-ilp (exp_libs/ilp.so)
# against the default schedule (exp_libs/cur.so): field kernel tests on the new library,
# then alternating bench pairs (both numerics' dominant kernels in the `kernels` digest).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g41; mkdir -p $O
ANR_HIP_LIB=$PWD/exp_libs/ilp.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_ingp_oracle_gpu.py -k "field or bench_size" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2 3; do
for v in ilp cur; do
ANR_HIP_LIB=$PWD/exp_libs/$v.so timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-numerics > $O/${v}_$rep.json.log 2>&1 || { tail -20 $O/${v}_$rep.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/${v}_$rep.json.log "$v rep $rep"
done
done
for v in ilp cur; do
ANR_HIP_LIB=$PWD/exp_libs/$v.so timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-numerics --numerics build > $O/${v}_build.json.log 2>&1 || { tail -20 $O/${v}_build.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/${v}_build.json.log "$v build"
done
