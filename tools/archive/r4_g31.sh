set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ANR_BENCH_DEBUG=1 timeout -k 10 400 python -u bench.py --steps 3 --no-cpu-baseline > gpurun_out/r4_g31.log 2>&1 || { tail -20 gpurun_out/r4_g31.log; exit 1; }
grep "count_hash" gpurun_out/r4_g31.log
