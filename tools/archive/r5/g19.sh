#!/bin/bash
# r5 close: SQ counter passes over the settled bench step, then the final bench lines:
# default (driver-style, with the CPU baseline), the surface-stream A/B, the per-rank
# 1,024-ray shape (hipGraph replay) and NeRF configs[1]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g19; mkdir -p $O
BENCH_ARGS=--no-alt-numerics bash tools/sq_bench.sh $O/sq > $O/sq.log 2>&1 || { tail -30 $O/sq.log; exit 1; }
python3 tools/pmc_table.py $O/sq > $O/sq_table.txt
rm -rf $O/sq/p1 $O/sq/p2 $O/sq/p3   # per-dispatch CSVs: too large to copy back
head -3 $O/sq_table.txt
timeout -k 10 500 python -u bench.py > $O/bench_default.json.log 2>&1 || { tail -30 $O/bench_default.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench_default.json.log default
ANR_SURFACE_STREAM=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-numerics > $O/bench_nosurf.json.log 2>&1 || { tail -30 $O/bench_nosurf.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench_nosurf.json.log surface_stream0
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-numerics > $O/bench_surf.json.log 2>&1 || { tail -30 $O/bench_surf.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench_surf.json.log surface_stream1
