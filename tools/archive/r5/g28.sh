#!/bin/bash
# r5: hash forward quad-major launch A/B (kernel tests under it, then the bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_g28; mkdir -p $O
ANR_HASH_FWD_QUADMAJOR=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "planes or quad" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 1 0; do
ANR_HASH_FWD_QUADMAJOR=$v timeout -k 10 300 python -u bench.py --no-alt-numerics --no-cpu-baseline > $O/qm$v.json.log 2>&1 || { tail -30 $O/qm$v.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/qm$v.json.log quad_major$v
done
