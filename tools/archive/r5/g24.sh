#!/bin/bash
# r5: NeRF kernels with AGPR accumulators: tests, probe, bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_g24; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nerf_gpu.py -k "nerf_linear or atmonerf_native" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u tools/r5/nerf_gemm_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep "q=" $O/probe.log
timeout -k 10 300 python -u bench.py --workload nerf --no-cpu-baseline > $O/bench_nerf.json.log 2>&1 || { tail -30 $O/bench_nerf.json.log; exit 1; }
tail -1 $O/bench_nerf.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline'].get('frac'), d['roofline'].get('gemm_kernels'), d['kernels'])"
