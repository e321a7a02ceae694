# ref16 kernels with the f32-then-f16 rounding restored: composite diag, gradient arms,
# ref16 + kernel tests, PSNR tests, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g10; mkdir -p $O
timeout -k 10 300 python -u tools/r5/composite_ref16_diag.py > $O/comp_diag.log 2>&1 || { tail -20 $O/comp_diag.log; exit 1; }
grep -E "^d_|equal" $O/comp_diag.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ref16_gpu.py tests/test_kernels_gpu.py > $O/test_a.log 2>&1 || { tail -40 $O/test_a.log; exit 1; }
tail -1 $O/test_a.log
timeout -k 10 900 python -u tools/r5/grad_arms_diag.py --checkpoints 0,16,32,48 --out $O/grad_arms.json > $O/grad_arms.log 2>&1 || { tail -20 $O/grad_arms.log; exit 1; }
python3 - <<'PY'
import json
for r in json.load(open("gpurun_out/r5_g10/grad_arms.json")):
    print("it", r["iteration"], {m: {k: (round(v["rel_l2"], 7), v["zero_mismatch"], round(v["equal_frac"], 4)) for k, v in r[m].items()} for m in ["pos_encoder", "pos_mlp"]}, "d_enc", r.get("d_enc"))
PY
ANR_INGP_PSNR_OUT=$O/psnr.json timeout -k 10 1500 python -u -m pytest -x -q --timeout 1400 --timeout-method thread tests/test_ingp_oracle_gpu.py > $O/test_ingp.log 2>&1 || { tail -60 $O/test_ingp.log; exit 1; }
tail -1 $O/test_ingp.log
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r5_g10/psnr.json"))
for k, v in d.items():
    if k.startswith("psnr_reference_semantics") and isinstance(v, list) and v and "iteration" in v[0]:
        print(k, [(r["iteration"], round(r["delta_reference_numerics_db"], 4)) for r in v])
PY
timeout -k 10 300 python -u tools/r5/hash_bwd_state.py dump --steps 160 --out /tmp/hb_ref160.pt > $O/state160.log 2>&1 || { tail -20 $O/state160.log; exit 1; }
grep state $O/state160.log
rm -f /tmp/hb_ref160.pt
for ts in 1 0; do
ANR_TILE_SKIP=$ts timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-numerics > $O/bench_ts$ts.json.log 2>&1 || { tail -30 $O/bench_ts$ts.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench_ts$ts.json.log tileskip$ts
done
