# ref16 composite timing + bit-exact tests; per-rank graphed step trace; reference-numerics
# step trace; extract throughput line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_b1024_trace gpurun_out/r4_ref_trace
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ref16_gpu.py > gpurun_out/r4_ref16_test2.log 2>&1 || { tail -30 gpurun_out/r4_ref16_test2.log; exit 1; }
tail -2 gpurun_out/r4_ref16_test2.log
timeout -k 10 120 python -u tools/ref16_bench.py > gpurun_out/r4_ref16_bench.log 2>&1 && cat gpurun_out/r4_ref16_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_b1024_trace -o run --output-format csv -- python3 bench.py --batch 1024 --graph on --steps 20 --warmup 10 --no-cpu-baseline --no-alt-numerics --no-kernel-timer --spec-peaks > gpurun_out/r4_b1024_trace/trace.log 2>&1 || { tail -20 gpurun_out/r4_b1024_trace/trace.log; exit 1; }
python tools/step_timeline.py gpurun_out/r4_b1024_trace --steps 1 > gpurun_out/r4_b1024_timeline.txt 2>&1; cat gpurun_out/r4_b1024_timeline.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_ref_trace -o run --output-format csv -- python3 bench.py --numerics reference --steps 5 --warmup 5 --no-cpu-baseline --no-alt-numerics --no-kernel-timer --spec-peaks > gpurun_out/r4_ref_trace/trace.log 2>&1 || { tail -20 gpurun_out/r4_ref_trace/trace.log; exit 1; }
python tools/step_timeline.py gpurun_out/r4_ref_trace --steps 1 > gpurun_out/r4_ref_timeline.txt 2>&1; cat gpurun_out/r4_ref_timeline.txt
timeout -k 10 300 python -u bench.py --workload extract --steps 20 --cpu-budget 15 > gpurun_out/r4_extract.json.log 2>&1 && tail -c 1500 gpurun_out/r4_extract.json.log
