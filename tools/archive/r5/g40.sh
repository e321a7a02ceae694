#!/bin/bash
# r5: hash-grid backward prefetch batch of 4 / 6 samples (exp_libs/bs4.so, bs6.so: no SGPR
# spills) against 8 (exp_libs/cur.so: 40 spilled SGPRs, ~424 v_readlane in the kernel):
# hash tests on bs4, then alternating bench lines, both numerics
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g40; mkdir -p $O
for v in bs4 bs6; do
ANR_HIP_LIB=$PWD/exp_libs/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "hashgrid and not tiles" > $O/test_$v.log 2>&1 || { tail -40 $O/test_$v.log; exit 1; }
echo "$v: $(tail -1 $O/test_$v.log)"
done
for rep in 1 2; do
for v in bs4 cur bs6; do
ANR_HIP_LIB=$PWD/exp_libs/$v.so timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-numerics > $O/${v}_$rep.json.log 2>&1 || { tail -20 $O/${v}_$rep.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/${v}_$rep.json.log "$v rep $rep"
done
done
for v in bs4 cur; do
ANR_HIP_LIB=$PWD/exp_libs/$v.so timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-numerics --numerics build > $O/${v}_build.json.log 2>&1 || { tail -20 $O/${v}_build.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/${v}_build.json.log "$v build"
done
