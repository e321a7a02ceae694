#!/bin/bash
# r5: hash-grid backward skip mode A/B under the build numerics
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_g21; mkdir -p $O
for m in 0 1 2; do
ANR_HASH_SKIP0=$m timeout -k 10 300 python -u bench.py --numerics build --no-alt-numerics --no-cpu-baseline > $O/build_skip$m.json.log 2>&1 || { tail -30 $O/build_skip$m.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/build_skip$m.json.log build_skip$m
done
