set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g9; mkdir -p $O
timeout -k 10 900 python -u tools/r5/grad_arms_diag.py --checkpoints 0 --out $O/grad_arms.json > $O/grad_arms.log 2>&1 || { tail -30 $O/grad_arms.log; exit 1; }
python3 - <<'PY'
import json
for r in json.load(open("gpurun_out/r5_g9/grad_arms.json")):
    print("it", r["iteration"], "d_enc", r.get("d_enc"))
    print("  d_sigma", r.get("d_sigma"))
    print("  d_color", r.get("d_color"))
    print("  top rows", [(t["row"], t["sample"]) for t in r.get("d_enc_top_rows", [])])
PY
