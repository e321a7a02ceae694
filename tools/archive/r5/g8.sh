# ref16 backward with the subnormal split of the input-gradient operands: tests, gradient
# arms, PSNR (split vs no-split library), bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g8; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ref16_gpu.py tests/test_kernels_gpu.py -k "field or ref16 or hash" > $O/test_a.log 2>&1 || { tail -40 $O/test_a.log; exit 1; }
tail -1 $O/test_a.log
timeout -k 10 900 python -u tools/r5/grad_arms_diag.py --out $O/grad_arms.json > $O/grad_arms.log 2>&1 || { tail -20 $O/grad_arms.log; exit 1; }
python3 - <<'PY'
import json
for r in json.load(open("gpurun_out/r5_g8/grad_arms.json")):
    print("it", r["iteration"], {m: {k: (round(v["rel_l2"], 7), v["zero_mismatch"], round(v["equal_frac"], 4)) for k, v in r[m].items()} for m in ["pos_encoder", "pos_mlp", "dir_mlp"]})
PY
ANR_INGP_PSNR_OUT=$O/psnr_split.json timeout -k 10 1500 python -u -m pytest -x -q --timeout 1400 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "psnr or reference_numerics" > $O/test_psnr_split.log 2>&1 || { tail -60 $O/test_psnr_split.log; exit 1; }
tail -1 $O/test_psnr_split.log
ANR_HIP_LIB=$PWD/exp_libs/libanr_nosplit.so ANR_INGP_PSNR_OUT=$O/psnr_nosplit.json timeout -k 10 1500 python -u -m pytest -x -q --timeout 1400 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "psnr_vs_reference and 1024" > $O/test_psnr_nosplit.log 2>&1 || { tail -60 $O/test_psnr_nosplit.log; exit 1; }
tail -1 $O/test_psnr_nosplit.log
python3 - <<'PY'
import json
for tag in ("split", "nosplit"):
    d = json.load(open(f"gpurun_out/r5_g8/psnr_{tag}.json"))
    for k, v in d.items():
        if k.startswith("psnr_reference_semantics") and isinstance(v, list) and v and "iteration" in v[0]:
            print(tag, k, [(r["iteration"], round(r["delta_reference_numerics_db"], 4)) for r in v])
PY
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json.log 2>&1 || { tail -30 $O/bench.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench.json.log split
