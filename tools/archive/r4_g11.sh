# hash bwd chunk length on the real bench coordinates (alternating, same box), then the
# headline rocprof passes (kernel trace + PMC) for profiles/r04_close
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
  for KB in 256 512; do
    ANR_HASH_KB=$KB timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-alt-numerics --numerics build > gpurun_out/r4_kab_${KB}_${rep}.json.log 2>&1 || exit 1
    python - <<PY
import json
l=[x for x in open("gpurun_out/r4_kab_${KB}_${rep}.json.log") if x.startswith("{")][-1]; d=json.loads(l)
r=d["roofline"]; print("KB ${KB} rep ${rep}", d["ms_per_step"], r["avg_ms"], r.get("atomic_requests_per_sample"), r["frac"])
PY
  done
done
