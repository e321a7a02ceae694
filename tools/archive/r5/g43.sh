#!/bin/bash
# r5 final (field kernels with the max-ILP scheduler): bench lines (driver-style default with the CPU baseline,
# the per-rank 1,024-ray shape, NeRF configs[1]), then the full GPU suite and smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g43; mkdir -p $O
timeout -k 10 500 python -u bench.py > $O/bench_default.json.log 2>&1 || { tail -30 $O/bench_default.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench_default.json.log default
timeout -k 10 400 python -u bench.py --batch 1024 --no-cpu-baseline > $O/bench_b1024.json.log 2>&1 || { tail -30 $O/bench_b1024.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench_b1024.json.log b1024
timeout -k 10 400 python -u bench.py --workload nerf > $O/bench_nerf.json.log 2>&1 || { tail -30 $O/bench_nerf.json.log; exit 1; }
tail -1 $O/bench_nerf.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('nerf', d['ms_per_step'], d['value'], d['roofline'].get('frac'), d['roofline'].get('gemm_kernels'))"
ANR_PSNR_OUT=$O/psnr_nerf.json ANR_INGP_PSNR_OUT=$O/psnr.json timeout -k 10 1000 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests -m gpu > $O/test_gpu.log 2>&1 || { tail -60 $O/test_gpu.log; exit 1; }
tail -1 $O/test_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
