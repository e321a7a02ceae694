# fma-mix scans, f16-input composite backward, extract run-length hint
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ref16_gpu.py tests/test_extract_gpu.py tests/test_pipeline_gpu.py > gpurun_out/r4_g19_test.log 2>&1 || { tail -30 gpurun_out/r4_g19_test.log; exit 1; }
tail -2 gpurun_out/r4_g19_test.log
for R in 1 2 4; do
  echo "R=$R" >> gpurun_out/r4_ref16M_bench.log
  ANR_REF16_R=$R timeout -k 10 120 python -u tools/ref16_bench.py >> gpurun_out/r4_ref16M_bench.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r4_ref16M_bench.log
timeout -k 10 300 python -u bench.py --workload extract --no-cpu-baseline > gpurun_out/r4_extract_runs.json.log 2>&1 || exit 1
grep '^{' gpurun_out/r4_extract_runs.json.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('extract', d['value'], d['ms_per_step'], d['kernels']['hash_fwd'])"
