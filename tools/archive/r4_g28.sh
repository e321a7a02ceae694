# reference numerics from a build-numerics warm start (alive field): headline + skip0 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
show() {
python3 - "$1" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l); r = d["roofline"] or {}; a = d.get("alt_numerics") or {}
print(sys.argv[1].split("/")[-1], d["numerics"], d["value"], d["ms_per_step"], "warm", d.get("warm_start"), "dEnc!=0", d.get("d_enc_nonzero_frac"),
      "| roof", r.get("kernel"), r.get("frac"), r.get("avg_ms"), r.get("atomic_requests_per_sample"),
      "| alt", a.get("numerics"), a.get("value"), a.get("ms_per_step"), a.get("d_enc_nonzero_frac"), a.get("warm_start"))
PY
}
timeout -k 10 500 python -u bench.py --no-cpu-baseline > gpurun_out/r4_g28_default.json.log 2>&1 || { tail -20 gpurun_out/r4_g28_default.json.log; exit 1; }
show gpurun_out/r4_g28_default.json.log
for rep in 1 2; do for S in 0 1; do
  ANR_HASH_SKIP0=$S timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-alt-numerics > gpurun_out/r4_g28_s${S}_${rep}.json.log 2>&1 || exit 1
  show gpurun_out/r4_g28_s${S}_${rep}.json.log
done; done
