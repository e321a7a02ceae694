set -o pipefail
O=gpurun_out/r2f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "hashgrid" --timeout 300 --timeout-method thread > $O/pytest_hash.log 2>&1 || exit $?
for m in 0 4; do
  ANR_HASHGRID_MODE=$m timeout -k 10 120 python -u tools/hash_probe.py --iters 5 > $O/probe_mode$m.log 2>&1 || exit $?
done
echo done
