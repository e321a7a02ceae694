#!/bin/bash
# r5: NeRF 128x128 wave tiles (ANR_NERF_BIG=1, P = 256 layers): tests + probe
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_g25; mkdir -p $O
ANR_NERF_BIG=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nerf_gpu.py -k "nerf_linear or atmonerf_native" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
ANR_NERF_BIG=1 timeout -k 10 300 python -u tools/r5/nerf_gemm_probe.py 256x256 76x256 > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep "q=" $O/probe.log
