# extract workload: hash forward chunk length / walker sweep (the extract grid's points
# are 250 m apart in altitude: far less corner reuse along a chunk than a ray's samples)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --workload extract --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r4_ex_$name.json.log 2>&1 || return 1
  python - "$name" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/r4_ex_{sys.argv[1]}.json.log") if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[1], round(d["value"] / 1e9, 3), "Gpts/s", d["ms_per_step"], "ms", "hash_fwd", d["kernels"]["hash_fwd"]["avg_ms"])
PY
}
run default ANR_X=0 && run kf1 ANR_HASH_KF=1 && run kf4 ANR_HASH_KF=4 && run kf9 ANR_HASH_KF=9 && run kf81 ANR_HASH_KF=81 && run v1 ANR_HASHGRID_MODE=6 ANR_HASH_KF=1 && run v1k8 ANR_HASHGRID_MODE=6 ANR_HASH_KF=8
