#!/bin/bash
# r6: NeRF hybrid arms (which kernel carries the configs[1] PSNR offset), paired cold-start
# liveness at batch 128, the INGP N=1024 oracle with f32 masters (dirs-ulp seeds) and 16 GPU
# replicas at the PSNR test's checkpoints
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g2; mkdir -p $O
timeout -k 10 400 python -u tools/nerf_hybrid_arms.py --mlp-accuracy --seeds 5 --out $O/nerf_hybrid.json > $O/nerf_hybrid.log 2>&1 || { tail -30 $O/nerf_hybrid.log; exit 1; }
timeout -k 10 400 python -u tools/liveness_paired.py --batch 128 --steps 30 --out $O/live_b128.json > $O/live_b128.log 2>&1 || { tail -30 $O/live_b128.log; exit 1; }
timeout -k 10 200 python -u tools/r5/gpu_psnr_repeat.py --samples 1024 --batch 64 --runs 16 --out $O/gpu_rep16.json > $O/gpu_rep16.log 2>&1 || { tail -30 $O/gpu_rep16.log; exit 1; }
timeout -k 10 700 python -u tools/ingp_oracle_spread.py --samples 1024 --batch 64 --checkpoints 0,8,32,48,64 --scene-device cuda --perturb dirs --runs 3 --master f32 --threads 16 --out $O/oracle_f32m.json > $O/oracle_f32m.log 2>&1 || { tail -30 $O/oracle_f32m.log; exit 1; }
