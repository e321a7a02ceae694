set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ANR_BENCH_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-alt-numerics > gpurun_out/r4_g25.log 2>&1 || { tail -20 gpurun_out/r4_g25.log; exit 1; }
grep "count_hash" gpurun_out/r4_g25.log
ANR_BENCH_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-alt-numerics --numerics build > gpurun_out/r4_g25b.log 2>&1 || { tail -20 gpurun_out/r4_g25b.log; exit 1; }
grep "count_hash" gpurun_out/r4_g25b.log
