#!/bin/bash
# Two ranks on the one GPU of a gpurun box over gloo (the RCCL path needs a GPU per rank):
# the overlapped and the plain gradient all-reduce, then the default single-GPU bench.
set -o pipefail
OUT=${1:-gpurun_out/dist}
mkdir -p "$OUT"
export ANR_DIST_BACKEND=gloo
for mode in overlap plain; do
  extra=""
  [ "$mode" = plain ] && extra="--no-overlap"
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 \
    --no-cpu-baseline --no-kernel-timer $extra > "$OUT/b2_$mode.log" 2>&1 || exit $?
done
unset ANR_DIST_BACKEND
timeout -k 10 300 python -u bench.py > "$OUT/b1.log" 2>&1 || exit $?
echo done
