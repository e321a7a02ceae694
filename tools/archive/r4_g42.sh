# hash bwd: flushes as range-checked buffer atomics (no divergent branch per corner, v1)
# vs HEAD's conditional global atomics (v0 = abso/libanr_hip_base.so); tests, then
# alternating bench pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_pipeline_gpu.py tests/test_ingp_oracle_gpu.py > gpurun_out/r4_g42_test.log 2>&1 || { tail -40 gpurun_out/r4_g42_test.log; exit 1; }
tail -1 gpurun_out/r4_g42_test.log
for rep in 1 2; do
for v in 0 1; do
if [ $v = 0 ]; then export ANR_HIP_LIB=$PWD/abso/libanr_hip_base.so; else unset ANR_HIP_LIB; fi
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r4_g42_v${v}_$rep.json.log 2>&1 || exit 1
python3 - $v $rep <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/r4_g42_v{sys.argv[1]}_{sys.argv[2]}.json.log") if x.startswith("{")][-1]
d = json.loads(l); r = d["roofline"]; a = d["alt_numerics"]
print("variant", sys.argv[1], "ref", d["value"], d["ms_per_step"], "| build", a["ms_per_step"], "| hash_bwd live", r["avg_ms"], r["frac"], r.get("atomic_requests_before_after"), "| field_bwd", d["kernels"]["field_bwd"]["avg_ms"], "hash_bwd", d["kernels"]["hash_bwd"]["avg_ms"])
PY
done
done
