#!/bin/bash
# r6: the whole GPU suite on the current library (durations recorded)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g14; mkdir -p $O
ANR_PSNR_OUT=$O/psnr_nerf.json ANR_INGP_PSNR_OUT=$O/psnr.json timeout -k 10 1140 python -u -m pytest tests -m gpu -x -q --timeout 1000 --timeout-method thread --durations=25 > $O/test_gpu.log 2>&1 || { tail -40 $O/test_gpu.log; exit 1; }
tail -n 32 $O/test_gpu.log
