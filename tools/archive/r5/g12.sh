#!/bin/bash
# r5: the NeRF dense-layer kernels (tests + bench line), the PSNR test with the
# chaos-horizon replicas, then the close-of-round rocprof trace + PMC traffic passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g12; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_nerf_gpu.py -s -k "nerf_linear or atmonerf_native" > $O/test_nerf_mlp.log 2>&1 || { tail -60 $O/test_nerf_mlp.log; exit 1; }
tail -15 $O/test_nerf_mlp.log
grep "rel L2" $O/test_nerf_mlp.log || true
timeout -k 10 300 python -u tools/r5/nerf_gemm_probe.py > $O/nerf_gemm_probe.log 2>&1 || { tail -30 $O/nerf_gemm_probe.log; exit 1; }
cat $O/nerf_gemm_probe.log
timeout -k 10 300 python -u bench.py --workload nerf --no-cpu-baseline > $O/bench_nerf.json.log 2>&1 || { tail -30 $O/bench_nerf.json.log; exit 1; }
tail -1 $O/bench_nerf.json.log
ANR_NERF_MLP=torch timeout -k 10 300 python -u bench.py --workload nerf --no-cpu-baseline > $O/bench_nerf_lib.json.log 2>&1 || { tail -30 $O/bench_nerf_lib.json.log; exit 1; }
tail -1 $O/bench_nerf_lib.json.log | cut -c1-300
ANR_INGP_PSNR_OUT=$O/psnr.json timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_ingp_oracle_gpu.py -k psnr_vs_reference > $O/test_psnr.log 2>&1 || { tail -60 $O/test_psnr.log; exit 1; }
tail -3 $O/test_psnr.log
BENCH_ARGS=--no-alt-numerics STEPS=5 bash tools/prof.sh $O/prof > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
