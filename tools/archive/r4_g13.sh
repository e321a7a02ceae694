# ref16 composite: wave-sync + one-segment-ahead prefetch, exp parked for pass 2; R sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ref16_gpu.py > gpurun_out/r4_ref16P_test.log 2>&1 || { tail -30 gpurun_out/r4_ref16P_test.log; exit 1; }
tail -2 gpurun_out/r4_ref16P_test.log
for R in 1 2 4; do
  echo "R=$R" >> gpurun_out/r4_ref16P_bench.log
  ANR_REF16_R=$R timeout -k 10 120 python -u tools/ref16_bench.py >> gpurun_out/r4_ref16P_bench.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r4_ref16P_bench.log
