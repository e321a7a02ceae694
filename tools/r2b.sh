set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r2b/bench.log 2>&1 || exit $?
bash tools/pmc_atomic.sh r2b/pmc || exit $?
echo done
