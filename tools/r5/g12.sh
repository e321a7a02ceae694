#!/bin/bash
# r5: the PSNR test with the chaos-horizon replicas, then the close-of-round rocprof
# trace + PMC traffic passes and the SQ counter passes over the settled bench step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g12; mkdir -p $O
ANR_INGP_PSNR_OUT=$O/psnr.json timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_ingp_oracle_gpu.py -k psnr_vs_reference > $O/test_psnr.log 2>&1 || { tail -60 $O/test_psnr.log; exit 1; }
tail -3 $O/test_psnr.log
BENCH_ARGS=--no-alt-numerics STEPS=5 bash tools/prof.sh $O/prof > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_nerf_gpu.py -k "nerf_linear or atmonerf_native" > $O/test_nerf_mlp.log 2>&1 || { tail -60 $O/test_nerf_mlp.log; exit 1; }
tail -15 $O/test_nerf_mlp.log
