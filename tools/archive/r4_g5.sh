set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -x -v --timeout 1000 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "psnr" > gpurun_out/r4_psnr.log 2>&1; rc=$?; tail -30 gpurun_out/r4_psnr.log; exit $rc
