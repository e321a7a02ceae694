set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g7; mkdir -p $O
timeout -k 10 500 python -u bench.py > $O/bench.json.log 2>&1 || { tail -30 $O/bench.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench.json.log new
timeout -k 10 900 python -u tools/r5/grad_arms_diag.py --out $O/grad_arms.json > $O/grad_arms.log 2>&1 || { tail -20 $O/grad_arms.log; exit 1; }
ANR_INGP_PSNR_OUT=$O/ingp_psnr.json timeout -k 10 1500 python -u -m pytest -x -v --timeout 1400 --timeout-method thread tests/test_ingp_oracle_gpu.py -k psnr > $O/test_psnr.log 2>&1 || { tail -60 $O/test_psnr.log; exit 1; }
grep -E "PASS|FAIL" $O/test_psnr.log | tail
