set -o pipefail
O=gpurun_out/r2g; mkdir -p $O
for m in 0 4; do
  ANR_HASHGRID_MODE=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline --spec-peaks > $O/bench_mode$m.log 2>&1 || exit $?
done
echo done
