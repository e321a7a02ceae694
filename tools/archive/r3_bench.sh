#!/bin/bash
# r03 bench lines on one GPU: the default (driver) line, the per-rank shape of 8-GPU strong
# scaling at a global batch of 8192 (1,024 rays per rank), the sharded optimizer at N=1,
# and a two-rank gloo rehearsal of the sharded optimizer on the one GPU.
# usage: tools/r3_bench.sh <out-dir>
set -o pipefail
OUT=${1:-gpurun_out/r3_bench}
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json.log" 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --batch 1024 --steps 50 --no-cpu-baseline \
  > "$OUT/bench_b1024.json.log" 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --shard-optimizer f16 --no-cpu-baseline \
  > "$OUT/bench_shard_f16.json.log" 2>&1 || exit $?
ANR_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
  --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timer --shard-optimizer f16 \
  > "$OUT/b2_gloo_shard_f16.json.log" 2>&1 || exit $?
echo done
