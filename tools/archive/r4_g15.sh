# N = 1,024 PSNR drift: FusedAdam vs f64 AdamW on tiny quantised gradients, then the
# gradient / optimizer split (oracle vs gpu vs hybrid)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/adam_tiny_grad_check.py --n 1000000 --steps 64 > gpurun_out/r4_adam_tiny.log 2>&1 || { tail -20 gpurun_out/r4_adam_tiny.log; exit 1; }
tail -5 gpurun_out/r4_adam_tiny.log
timeout -k 10 1000 python -u tools/psnr_hybrid_diag.py --iters 64 --every 8 --out gpurun_out/r4_psnr_hybrid.json > gpurun_out/r4_psnr_hybrid.log 2>&1 || { tail -20 gpurun_out/r4_psnr_hybrid.log; exit 1; }
tail -3 gpurun_out/r4_psnr_hybrid.log
