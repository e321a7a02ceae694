# hash bwd request-count instrument: its test, then the headline bench counting in-run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "hash" > gpurun_out/r4_g24_test.log 2>&1 || { tail -30 gpurun_out/r4_g24_test.log; exit 1; }
tail -1 gpurun_out/r4_g24_test.log
timeout -k 10 400 python -u bench.py > gpurun_out/r4_bench_g24.json.log 2>&1 || { tail -20 gpurun_out/r4_bench_g24.json.log; exit 1; }
python3 - <<'PY'
import json
l = [x for x in open("gpurun_out/r4_bench_g24.json.log") if x.startswith("{")][-1]
d = json.loads(l); r = d["roofline"]; a = d["alt_numerics"]
print("ref", d["value"], d["ms_per_step"], "| build", a["value"], a["ms_per_step"])
print({k: r.get(k) for k in ["kernel", "achieved", "peak", "frac", "avg_ms", "atomic_requests_per_launch", "atomic_requests_per_sample", "atomic_requests_source"]})
PY
