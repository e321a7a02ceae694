#!/bin/bash
# r5 close: the per-rank 1,024-ray shape (hipGraph replay) and NeRF configs[1]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g20; mkdir -p $O
timeout -k 10 400 python -u bench.py --batch 1024 --no-cpu-baseline > $O/bench_b1024.json.log 2>&1 || { tail -30 $O/bench_b1024.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench_b1024.json.log b1024
timeout -k 10 300 python -u bench.py --workload nerf > $O/bench_nerf.json.log 2>&1 || { tail -30 $O/bench_nerf.json.log; exit 1; }
tail -1 $O/bench_nerf.json.log | cut -c1-400
