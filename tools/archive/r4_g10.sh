# PSNR drift diagnostic at 1,024 samples per ray, then the default bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 60 python -u tools/f16_denorm_probe.py 2>&1 | tail -1
timeout -k 10 500 python -u tools/psnr_drift_diag.py --out gpurun_out/r4_psnr_drift.json > gpurun_out/r4_psnr_drift.log 2>&1 || { tail -20 gpurun_out/r4_psnr_drift.log; exit 1; }
tail -3 gpurun_out/r4_psnr_drift.log | cut -c1-200
timeout -k 10 400 python -u bench.py > gpurun_out/r4_bench_default.json.log 2>&1 && tail -c 300 gpurun_out/r4_bench_default.json.log || exit 1
timeout -k 10 300 python -u bench.py --batch 1024 --no-cpu-baseline > gpurun_out/r4_b1024_default.json.log 2>&1 && tail -c 300 gpurun_out/r4_b1024_default.json.log
