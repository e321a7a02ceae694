# driver-style headline run (cpu baseline included) on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r4_final_bench.json.log 2>&1 || { tail -20 gpurun_out/r4_final_bench.json.log; exit 1; }
python3 - <<'PY'
import json
l = [x for x in open("gpurun_out/r4_final_bench.json.log") if x.startswith("{")][-1]
d = json.loads(l); r = d["roofline"]; a = d["alt_numerics"]
print("ref", d["value"], d["ms_per_step"], d["d_enc_nonzero_frac"], d["warm_start"], "| build", a["value"], a["ms_per_step"])
print({k: r.get(k) for k in ["kernel", "bound", "achieved", "peak", "unit", "frac", "avg_ms", "atomic_requests_per_sample", "atomic_requests_before_after", "d_enc_nonzero_before_after", "traffic"]})
print("cpu", d["cpu_baseline"]["value"])
PY
