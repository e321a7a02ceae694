set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/psnr_gpu_self_spread.py --runs 3 --out gpurun_out/r4_psnr_self_spread.json > gpurun_out/r4_psnr_self_spread.log 2>&1 || { tail -20 gpurun_out/r4_psnr_self_spread.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_psnr_self_spread.log | tail -12
bash tools/r4_g17.sh
