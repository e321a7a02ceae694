set -o pipefail
O=gpurun_out/r2d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_f16.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --dtype bf16 > $O/bench_bf16.log 2>&1 || exit $?
bash tools/pmc_atomic.sh r2d/pmc || exit $?
echo done
