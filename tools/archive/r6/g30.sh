#!/bin/bash
# r6 final: the whole GPU suite, the driver-style bench lines + smoke (TAG=r06_final), then
# the rocprof kernel trace + PMC + SQ passes of the same library
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g30; mkdir -p $O
ANR_PSNR_OUT=$O/psnr_nerf.json ANR_INGP_PSNR_OUT=$O/psnr.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 800 --timeout-method thread --durations=15 > $O/test_gpu.log 2>&1 || { tail -40 $O/test_gpu.log; exit 1; }
tail -n 3 $O/test_gpu.log
TAG=r06_final bash tools/r6/final_bench.sh
