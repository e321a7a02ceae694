#!/bin/bash
# r5: NeRF NT kernel bound probe: normal / no operand loads / no MFMAs (256x256 only)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_g16; mkdir -p $O
for d in 0 1 3; do
ANR_NERF_DBG=$d timeout -k 10 200 python -u tools/r5/nerf_gemm_probe.py 256x256 76x256 > $O/dbg$d.log 2>&1 || { tail -20 $O/dbg$d.log; exit 1; }
echo "DBG=$d"; grep "q=" $O/dbg$d.log
done
