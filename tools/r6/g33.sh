#!/bin/bash
# r6 close: the whole GPU suite and the driver-style bench lines + smoke (TAG=r06_close) on
# the library with the list pass early exit
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g33; mkdir -p $O
ANR_PSNR_OUT=$O/psnr_nerf.json ANR_INGP_PSNR_OUT=$O/psnr.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 800 --timeout-method thread --durations=10 > $O/test_gpu.log 2>&1 || { tail -40 $O/test_gpu.log; exit 1; }
tail -n 3 $O/test_gpu.log
TAG=r06_close bash tools/r6/final_bench.sh
