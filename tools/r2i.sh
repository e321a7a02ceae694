set -o pipefail
O=gpurun_out/r2i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "hashgrid" --timeout 300 --timeout-method thread > $O/pytest_hash.log 2>&1 || exit $?
for m in 0 5; do
  ANR_HASHGRID_MODE=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline --spec-peaks > $O/bench_mode$m.log 2>&1 || exit $?
done
echo done
