#!/bin/bash
# r5: NeRF kernels on random vs all-zero operands (does the data set the MFMA rate?)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_g23; mkdir -p $O
timeout -k 10 200 python -u tools/r5/nerf_gemm_probe.py 256x256 > $O/rand.log 2>&1 || { tail -20 $O/rand.log; exit 1; }
timeout -k 10 200 python -u tools/r5/nerf_gemm_probe.py 256x256 --zeros > $O/zeros.log 2>&1 || { tail -20 $O/zeros.log; exit 1; }
echo random; grep "q=" $O/rand.log; echo zeros; grep "q=" $O/zeros.log
