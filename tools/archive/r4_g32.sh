# hash bwd zero-batch skip: hash tests, then reference-numerics A/B (skip0 on/off covers both skips)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "hash" > gpurun_out/r4_g32_test.log 2>&1 || { tail -30 gpurun_out/r4_g32_test.log; exit 1; }
tail -1 gpurun_out/r4_g32_test.log
show() {
python3 - "$1" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l); r = d["roofline"] or {}; a = d.get("alt_numerics") or {}
print(sys.argv[1].split("/")[-1], d["numerics"], d["value"], d["ms_per_step"], "dEnc!=0", d.get("d_enc_nonzero_frac"),
      "| roof", r.get("kernel"), r.get("frac"), r.get("avg_ms"), r.get("atomic_requests_per_sample"),
      "| alt", a.get("numerics"), a.get("ms_per_step"), "| hash_bwd", d["kernels"].get("hash_bwd", {}).get("avg_ms"))
PY
}
for rep in 1 2; do for S in 0 1; do
  ANR_HASH_SKIP0=$S timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r4_g32_s${S}_${rep}.json.log 2>&1 || exit 1
  show gpurun_out/r4_g32_s${S}_${rep}.json.log
done; done
