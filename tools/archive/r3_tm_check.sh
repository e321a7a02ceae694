set -o pipefail
tools/r3_run.sh gpurun_out/r4g "tests/test_tile_max_gpu.py" 300 "tests/test_kernels_gpu.py" 600 "tests/test_pipeline_gpu.py tests/test_ingp_oracle_gpu.py" 500 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/r4g/bench.log 2>&1
