#!/bin/bash
# r6: row-walker tests after the chunk rounding / in-place fallback, then the rocprof kernel
# trace + PMC + SQ passes of the current library (tools/r6/prof_final.sh, TAG=r06_c)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g24; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "rows or zero_color" > $O/test_kern.log 2>&1 || { tail -40 $O/test_kern.log; exit 1; }
tail -n 1 $O/test_kern.log
TAG=r06_c bash tools/r6/prof_final.sh > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
tail -3 $O/prof.log
