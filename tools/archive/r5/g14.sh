#!/bin/bash
# r5: NeRF dense-layer kernels v2 (buffer loads, prefetch ring, 16-B epilogue): tests,
# probe at prefetch depth 1 and 2, NeRF bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g14; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_nerf_gpu.py -k "nerf_linear or atmonerf_native" > $O/test_nerf_mlp.log 2>&1 || { tail -60 $O/test_nerf_mlp.log; exit 1; }
tail -3 $O/test_nerf_mlp.log
grep "rel L2" $O/test_nerf_mlp.log | head -2 || true
for pd in 1024 2048; do
ANR_NERF_BLOCKS=$pd timeout -k 10 300 python -u tools/r5/nerf_gemm_probe.py > $O/probe_pd$pd.log 2>&1 || { tail -30 $O/probe_pd$pd.log; exit 1; }
echo "BLOCKS=$pd"; grep "q=" $O/probe_pd$pd.log
done
timeout -k 10 300 python -u bench.py --workload nerf --no-cpu-baseline > $O/bench_nerf.json.log 2>&1 || { tail -30 $O/bench_nerf.json.log; exit 1; }
tail -1 $O/bench_nerf.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline'].get('frac'), d['roofline'].get('gemm_kernels'), d['kernels'])"
ANR_NERF_MLP=torch timeout -k 10 300 python -u bench.py --workload nerf --no-cpu-baseline > $O/bench_nerf_lib.json.log 2>&1 || { tail -30 $O/bench_nerf_lib.json.log; exit 1; }
tail -1 $O/bench_nerf_lib.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('library', d['ms_per_step'], d['value'], d['roofline'].get('frac'))"
