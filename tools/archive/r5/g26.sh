#!/bin/bash
# r5: GPU liveness from a cold start at the oracle_liveness batch (128 rays x 1,024),
# both numerics, beside tools/r5/oracle_liveness.py; then the NeRF bench line with the
# 128 x 128 tiles and the NeRF kernel tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_g26; mkdir -p $O
for n in reference build; do
timeout -k 10 200 python -u tools/liveness.py --numerics $n --batch 128 --steps 20 > $O/live_$n.log 2>&1 || { tail -20 $O/live_$n.log; exit 1; }
echo "== $n"; grep step $O/live_$n.log | cut -c1-110
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nerf_gpu.py > $O/test_nerf.log 2>&1 || { tail -40 $O/test_nerf.log; exit 1; }
tail -1 $O/test_nerf.log
timeout -k 10 300 python -u bench.py --workload nerf --no-cpu-baseline > $O/bench_nerf.json.log 2>&1 || { tail -30 $O/bench_nerf.json.log; exit 1; }
tail -1 $O/bench_nerf.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline'].get('frac'), d['roofline'].get('gemm_kernels'), d['kernels'])"
