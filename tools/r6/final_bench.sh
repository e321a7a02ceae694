#!/bin/bash
# r6 final: driver-style bench lines (configs[2] headline with the CPU baseline, the
# per-rank 1,024-ray shape, NeRF configs[1]) and smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06_final}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json.log 2>&1 || { tail -30 $O/bench.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench.json.log headline
timeout -k 10 300 python -u bench.py --batch 1024 --no-cpu-baseline --no-alt-numerics > $O/bench_b1024.json.log 2>&1 || { tail -30 $O/bench_b1024.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench_b1024.json.log b1024
timeout -k 10 300 python -u bench.py --workload nerf --no-cpu-baseline > $O/bench_nerf.json.log 2>&1 || { tail -30 $O/bench_nerf.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench_nerf.json.log nerf
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -n 3 $O/smoke.log
