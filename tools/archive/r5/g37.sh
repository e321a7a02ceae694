#!/bin/bash
# r5: NeRF dense layers with three operand stages (loads two k-steps ahead; ANR_NERF_STAGES=3,
# the default in this library) against the two-stage loop (ANR_NERF_STAGES=2): NeRF kernel
# tests under both, GEMM probe and NeRF bench under both
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g37; mkdir -p $O
for v in 3 2; do
ANR_NERF_STAGES=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nerf_gpu.py > $O/test_nerf_$v.log 2>&1 || { tail -40 $O/test_nerf_$v.log; exit 1; }
echo "stages $v: $(tail -1 $O/test_nerf_$v.log)"
done
for v in 3 2; do
ANR_NERF_STAGES=$v timeout -k 10 300 python -u tools/r5/nerf_gemm_probe.py > $O/probe_$v.log 2>&1 || { tail -20 $O/probe_$v.log; exit 1; }
echo "== probe stages $v"; grep "^q=" $O/probe_$v.log
done
for rep in 1 2; do
for v in 3 2; do
ANR_NERF_STAGES=$v timeout -k 10 300 python -u bench.py --workload nerf --no-cpu-baseline > $O/bench_nerf_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_nerf_${v}_$rep.json.log; exit 1; }
echo "== bench stages $v rep $rep: $(tail -1 $O/bench_nerf_${v}_$rep.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline'].get('frac'), d['roofline'].get('gemm_kernels', {}).get('ms_per_step'))")"
done
done
