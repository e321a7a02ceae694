#!/bin/bash
# r5: pin the N=1024 PSNR distance. GPU run-to-run spread of the reference-numerics
# pipeline, and the oracle's own spread in the PSNR test's exact configuration (scene
# built on the GPU), three perturbation kinds in parallel on the CPU.
set -o pipefail
O=gpurun_out/r5_g11; mkdir -p $O
timeout -k 10 300 python -u tools/r5/gpu_psnr_repeat.py --runs 4 --out $O/gpu_repeat.json > $O/gpu_repeat.log 2>&1 || { tail -30 $O/gpu_repeat.log; exit 1; }
cat $O/gpu_repeat.log
pids=()
for k in acc dirs gradnoise; do
  timeout -k 10 1000 python -u tools/ingp_oracle_spread.py --samples 1024 --batch 64 \
    --checkpoints 0,8,32,48,64 --perturb $k --runs 1 --threads 5 --scene-device cuda \
    --out $O/oracle_$k.json > $O/oracle_$k.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
tail -3 $O/oracle_*.log
exit $rc
