#!/bin/bash
# r5: NeRF operand stages, auto rule (ANR_NERF_STAGES unset = 0) vs forced 2 and 3:
# NeRF kernel tests under the auto rule, then GEMM probe and NeRF bench under each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g38; mkdir -p $O
for v in 0; do
ANR_NERF_STAGES=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nerf_gpu.py > $O/test_nerf_$v.log 2>&1 || { tail -40 $O/test_nerf_$v.log; exit 1; }
echo "stages $v: $(tail -1 $O/test_nerf_$v.log)"
done
for v in 0 2 3; do
ANR_NERF_STAGES=$v timeout -k 10 300 python -u tools/r5/nerf_gemm_probe.py > $O/probe_$v.log 2>&1 || { tail -20 $O/probe_$v.log; exit 1; }
echo "== probe stages $v"; grep "^q=" $O/probe_$v.log
done
for rep in 1 2; do
for v in 0 2 3; do
ANR_NERF_STAGES=$v timeout -k 10 300 python -u bench.py --workload nerf --no-cpu-baseline > $O/bench_nerf_${v}_$rep.json.log 2>&1 || { tail -30 $O/bench_nerf_${v}_$rep.json.log; exit 1; }
echo "== bench stages $v rep $rep: $(tail -1 $O/bench_nerf_${v}_$rep.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline'].get('frac'), d['roofline'].get('gemm_kernels', {}).get('ms_per_step'))")"
done
done
