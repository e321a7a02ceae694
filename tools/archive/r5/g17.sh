#!/bin/bash
# r5 close: the whole GPU test suite, then smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g17; mkdir -p $O
ANR_PSNR_OUT=$O/psnr_nerf.json ANR_INGP_PSNR_OUT=$O/psnr.json timeout -k 10 1000 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests -m gpu > $O/test_gpu.log 2>&1 || { tail -60 $O/test_gpu.log; exit 1; }
tail -3 $O/test_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
