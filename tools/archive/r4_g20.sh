# headline (reference numerics, build numerics alongside) and the per-rank 1,024-ray line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/r4_bench_g20.json.log 2>&1 || { tail -20 gpurun_out/r4_bench_g20.json.log; exit 1; }
timeout -k 10 300 python -u bench.py --batch 1024 --no-cpu-baseline > gpurun_out/r4_b1024_g20.json.log 2>&1 || exit 1
for f in r4_bench_g20 r4_b1024_g20; do
python3 - $f <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/{sys.argv[1]}.json.log") if x.startswith("{")][-1]
d = json.loads(l); a = d.get("alt_numerics") or {}
print(sys.argv[1], d["numerics"], d["value"], d["ms_per_step"], d.get("host_ms_per_step"), d.get("graph"), "| alt", a.get("numerics"), a.get("value"), a.get("ms_per_step"))
print({k: v["avg_ms"] for k, v in d.get("kernels", {}).items()})
PY
done
