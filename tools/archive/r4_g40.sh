# hash bwd: dL/dy rows staged through LDS (one 16-B load per lane per 8-sample batch) vs
# the 8 per-column loads; tests, then alternating bench pairs (ANR_HASH_LDS_ROWS=0 / 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_pipeline_gpu.py tests/test_ingp_oracle_gpu.py > gpurun_out/r4_g40_test.log 2>&1 || { tail -40 gpurun_out/r4_g40_test.log; exit 1; }
tail -1 gpurun_out/r4_g40_test.log
for rep in 1 2; do
for v in 0 1; do
ANR_HASH_LDS_ROWS=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r4_g40_lds${v}_$rep.json.log 2>&1 || exit 1
python3 - $v $rep <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/r4_g40_lds{sys.argv[1]}_{sys.argv[2]}.json.log") if x.startswith("{")][-1]
d = json.loads(l); r = d["roofline"]; a = d["alt_numerics"]
print("lds_rows", sys.argv[1], "ref", d["value"], d["ms_per_step"], "| build", a["ms_per_step"], "| hash_bwd live", r["avg_ms"], r["frac"], r.get("atomic_requests_before_after"), "| field_bwd", d["kernels"]["field_bwd"]["avg_ms"], "hash_bwd", d["kernels"]["hash_bwd"]["avg_ms"])
PY
done
done
