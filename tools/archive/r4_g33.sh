# r04 close profile (final tree): kernel trace + FETCH / WRITE / atomic PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BENCH_ARGS="--no-alt-numerics" bash tools/prof.sh gpurun_out/r04_close2
