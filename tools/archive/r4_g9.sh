# r04: ref16 kernels after the vectorised scans (bit-exact tests, timing), reference-numerics
# oracle steps + PSNR, then the default bench line (reference numerics headline, build alt)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ref16_gpu.py tests/test_graph_gpu.py > gpurun_out/r4_g9_test.log 2>&1 || { tail -30 gpurun_out/r4_g9_test.log; exit 1; }
tail -2 gpurun_out/r4_g9_test.log
timeout -k 10 120 python -u tools/ref16_bench.py > gpurun_out/r4_ref16_bench2.log 2>&1 && cat gpurun_out/r4_ref16_bench2.log || exit 1
export ANR_INGP_PSNR_OUT=gpurun_out/r4_ingp_oracle_records2.json
timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "reference" > gpurun_out/r4_ingp_ref.log 2>&1 || { tail -30 gpurun_out/r4_ingp_ref.log; exit 1; }
tail -6 gpurun_out/r4_ingp_ref.log
timeout -k 10 400 python -u bench.py > gpurun_out/r4_bench_default.json.log 2>&1 && tail -c 300 gpurun_out/r4_bench_default.json.log || exit 1
timeout -k 10 300 python -u bench.py --batch 1024 --no-cpu-baseline > gpurun_out/r4_b1024_default.json.log 2>&1 && tail -c 300 gpurun_out/r4_b1024_default.json.log
