#!/bin/bash
# r6: the whole GPU suite, then the driver-style bench lines and smoke (TAG=r06_d)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g25; mkdir -p $O
ANR_PSNR_OUT=$O/psnr_nerf.json ANR_INGP_PSNR_OUT=$O/psnr.json timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread --durations=15 > $O/test_gpu.log 2>&1 || { tail -40 $O/test_gpu.log; exit 1; }
tail -n 3 $O/test_gpu.log
TAG=r06_d bash tools/r6/final_bench.sh
