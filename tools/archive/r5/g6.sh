# ref16 exponent-shifted MFMA operands + quad-plane enc: parity tests, probe, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g6; mkdir -p $O
timeout -k 10 120 python -u tools/r5/hash_fwd_planes_probe.py > $O/planes.log 2>&1 || { tail -20 $O/planes.log; exit 1; }
tail -1 $O/planes.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ref16_gpu.py tests/test_graph_gpu.py tests/test_kernels_gpu.py tests/test_pipeline_gpu.py > $O/test_a.log 2>&1 || { tail -40 $O/test_a.log; exit 1; }
tail -1 $O/test_a.log
ANR_INGP_PSNR_OUT=$O/ingp_records.json timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ingp_oracle_gpu.py -k "not psnr" > $O/test_ingp.log 2>&1 || { tail -60 $O/test_ingp.log; exit 1; }
tail -1 $O/test_ingp.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json.log 2>&1 || { tail -30 $O/bench.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench.json.log new
