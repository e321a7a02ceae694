set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ref16_field_diag.py --samples 1024 --rays 64 --psnr-batch > gpurun_out/r4_field_diag_1024.log 2>&1 || { tail -20 gpurun_out/r4_field_diag_1024.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_field_diag_1024.log | head -120
