# ref16 composite with R rays per wavefront: bit-exact tests, R sweep of the two kernels,
# then the headline bench (reference numerics)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ref16_gpu.py > gpurun_out/r4_ref16R_test.log 2>&1 || { tail -30 gpurun_out/r4_ref16R_test.log; exit 1; }
tail -2 gpurun_out/r4_ref16R_test.log
for R in 1 2 4 8; do
  echo "R=$R" >> gpurun_out/r4_ref16R_bench.log
  ANR_REF16_R=$R timeout -k 10 120 python -u tools/ref16_bench.py >> gpurun_out/r4_ref16R_bench.log 2>&1 || exit 1
done
cat gpurun_out/r4_ref16R_bench.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4_bench_ref16R.json.log 2>&1 || exit 1
python - <<'PY'
import json
l=[x for x in open("gpurun_out/r4_bench_ref16R.json.log") if x.startswith("{")][-1]; d=json.loads(l)
print("ref", d["ms_per_step"], d["value"], "alt", d["alt_numerics"]["ms_per_step"])
print(json.dumps(d.get("kernels", {}))[:1500])
PY
