# per-rank line (reference numerics from the warm start), then the full GPU suite and smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --batch 1024 --no-cpu-baseline > gpurun_out/r4_b1024_alive.json.log 2>&1 || { tail -20 gpurun_out/r4_b1024_alive.json.log; exit 1; }
python3 - <<'PY'
import json
l = [x for x in open("gpurun_out/r4_b1024_alive.json.log") if x.startswith("{")][-1]
d = json.loads(l); a = d["alt_numerics"]
print("b1024", d["numerics"], d["value"], d["ms_per_step"], d["host_ms_per_step"], d["graph"], d["d_enc_nonzero_frac"], "| alt", a["numerics"], a["value"], a["ms_per_step"])
print({k: v["avg_ms"] for k, v in d["kernels"].items()})
PY
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 1200 --timeout-method thread > gpurun_out/r4_gpu_suite.log 2>&1 || { tail -40 gpurun_out/r4_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r4_gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -3 gpurun_out/r4_smoke.log
