#!/bin/bash
# r5: hash forward v10 (planes, level-pipelined): kernel tests at AHEAD = 1 (default) and 2,
# then alternating bench lines ANR_HASH_FWD_PIPE = 1 / 0 (v9) / 2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g32; mkdir -p $O
for p in 1 2; do
ANR_HASH_FWD_PIPE=$p timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "outside_grid or quad_planes or bench_size" > $O/test_p$p.log 2>&1 || { tail -30 $O/test_p$p.log; exit 1; }
echo "pipe $p: $(tail -1 $O/test_p$p.log)"
done
for rep in 1 2; do
for p in 1 0 2; do
ANR_HASH_FWD_PIPE=$p timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/p${p}_$rep.json.log 2>&1 || { tail -30 $O/p${p}_$rep.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/p${p}_$rep.json.log "pipe $p rep $rep"
done
done
