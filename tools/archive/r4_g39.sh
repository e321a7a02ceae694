# final tree after the scalar-coordinate hash bwd: GPU suite, smoke, close profile
# (kernel trace + PMC passes, summarised on the box so the bench reads the new traffic),
# then the driver-style headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_gpu_suite_final.log 2>&1 || { tail -40 gpurun_out/r4_gpu_suite_final.log; exit 1; }
tail -1 gpurun_out/r4_gpu_suite_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke_final.log 2>&1 || { tail -20 gpurun_out/r4_smoke_final.log; exit 1; }
tail -1 gpurun_out/r4_smoke_final.log
BENCH_ARGS="--no-alt-numerics" bash tools/prof.sh gpurun_out/r04_close3 || exit 1
python3 tools/prof_summary.py gpurun_out/r04_close3 r04_close > gpurun_out/r04_close3_summary.log 2>&1 || { tail gpurun_out/r04_close3_summary.log; exit 1; }
mkdir -p gpurun_out/r04_close3_profiles && cp profiles/pmc_traffic.json profiles/r04_close_summary.md profiles/r04_close_kernel_stats.csv gpurun_out/r04_close3_profiles/
timeout -k 10 600 python -u bench.py > gpurun_out/r4_final_bench.json.log 2>&1 || { tail -20 gpurun_out/r4_final_bench.json.log; exit 1; }
python3 - <<'PY'
import json
l = [x for x in open("gpurun_out/r4_final_bench.json.log") if x.startswith("{")][-1]
d = json.loads(l); r = d["roofline"]; a = d["alt_numerics"]
print("ref", d["value"], d["ms_per_step"], d["d_enc_nonzero_frac"], d["warm_start"], "| build", a["value"], a["ms_per_step"])
print({k: r.get(k) for k in ["kernel", "bound", "achieved", "peak", "unit", "frac", "avg_ms", "atomic_requests_per_sample", "atomic_requests_before_after", "d_enc_nonzero_before_after", "traffic"]})
print("cpu", d["cpu_baseline"]["value"])
PY
