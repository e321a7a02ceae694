#!/bin/bash
# r6: NeRF configs[1] offset -- render check (native vs library forward on the same trained
# weights), MLP gradient accuracy vs f64 (same upstream gradient), hidden-unit permutation
# arms (8 summation orders, native / library / oracle); then paired liveness at batch 1,024
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_g3; mkdir -p $O
timeout -k 10 700 python -u tools/nerf_hybrid_arms.py --render-check --mlp-accuracy --seeds 0 --perms 8 --out $O/nerf_perm.json > $O/nerf_perm.log 2>&1 || { tail -30 $O/nerf_perm.log; exit 1; }
timeout -k 10 450 python -u tools/liveness_paired.py --batch 1024 --steps 30 --arms oracle_f32_master --out $O/live_b1024.json > $O/live_b1024.log 2>&1 || { tail -30 $O/live_b1024.log; exit 1; }
