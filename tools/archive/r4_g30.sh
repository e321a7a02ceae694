# deferred tcnn gradient rounding in AdamW: equality test, Adam kernel tests, then the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "deferred or step_reference or f16_gradient" tests/test_kernels_gpu.py -k "adam or deferred or step_reference or f16_gradient" > gpurun_out/r4_g30_test.log 2>&1 || { tail -30 gpurun_out/r4_g30_test.log; exit 1; }
tail -1 gpurun_out/r4_g30_test.log
timeout -k 10 500 python -u bench.py --no-cpu-baseline > gpurun_out/r4_g30_bench.json.log 2>&1 || { tail -20 gpurun_out/r4_g30_bench.json.log; exit 1; }
python3 - <<'PY'
import json
l = [x for x in open("gpurun_out/r4_g30_bench.json.log") if x.startswith("{")][-1]
d = json.loads(l); a = d["alt_numerics"]; r = d["roofline"]
print("ref", d["value"], d["ms_per_step"], d["d_enc_nonzero_frac"], "| build", a["value"], a["ms_per_step"], "| roof", r["kernel"], r["frac"], r["avg_ms"])
print({k: v["avg_ms"] for k, v in d["kernels"].items()})
PY
