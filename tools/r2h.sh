set -o pipefail
O=gpurun_out/r2h; mkdir -p $O
export TMPDIR=/tmp
bash tools/sq_bench.sh $O/sq || exit $?
timeout -k 10 300 python -u bench.py --variant committed --no-cpu-baseline > $O/bench_committed.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload nerf > $O/bench_nerf.log 2>&1 || exit $?
echo done
