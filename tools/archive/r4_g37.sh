# f16 dL/denc in reference numerics: oracle / pipeline / kernel tests, then the bench twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ingp_oracle_gpu.py tests/test_ref16_gpu.py tests/test_pipeline_gpu.py > gpurun_out/r4_g37_test.log 2>&1 || { tail -40 gpurun_out/r4_g37_test.log; exit 1; }
tail -1 gpurun_out/r4_g37_test.log
for rep in 1 2; do
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r4_g37_bench_$rep.json.log 2>&1 || exit 1
python3 - $rep <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/r4_g37_bench_{sys.argv[1]}.json.log") if x.startswith("{")][-1]
d = json.loads(l); r = d["roofline"]; a = d["alt_numerics"]
print("ref", d["value"], d["ms_per_step"], "| build", a["ms_per_step"], "| hash_bwd live", r["avg_ms"], r["frac"], r.get("atomic_requests_before_after"), "| field_bwd", d["kernels"]["field_bwd"]["avg_ms"], "hash_bwd", d["kernels"]["hash_bwd"]["avg_ms"])
PY
done
