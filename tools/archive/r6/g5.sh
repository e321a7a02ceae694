#!/bin/bash
# r6: INGP N=1024 GPU replica distribution at 64 iterations in the test's company: with a
# build-numerics pipeline interleaved, with the surface branch on the main stream, with the
# oracle interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g5; mkdir -p $O
timeout -k 10 200 python -u tools/r5/gpu_psnr_repeat.py --samples 1024 --batch 64 --runs 16 --with-build --out $O/rep_build.json > $O/rep_build.log 2>&1 || { tail -30 $O/rep_build.log; exit 1; }
timeout -k 10 200 python -u tools/r5/gpu_psnr_repeat.py --samples 1024 --batch 64 --runs 16 --no-surface-stream --out $O/rep_nosurf.json > $O/rep_nosurf.log 2>&1 || { tail -30 $O/rep_nosurf.log; exit 1; }
timeout -k 10 200 python -u tools/r5/gpu_psnr_repeat.py --samples 1024 --batch 64 --runs 16 --out $O/rep_plain.json > $O/rep_plain.log 2>&1 || { tail -30 $O/rep_plain.log; exit 1; }
timeout -k 10 400 python -u tools/r5/gpu_psnr_repeat.py --samples 1024 --batch 64 --runs 8 --with-build --with-oracle --out $O/rep_oracle.json > $O/rep_oracle.log 2>&1 || { tail -30 $O/rep_oracle.log; exit 1; }
