# r04 close profile: kernel trace + FETCH / WRITE / atomic PMC passes of the headline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BENCH_ARGS="--no-alt-numerics" bash tools/prof.sh gpurun_out/r04_close && python3 tools/prof_summary.py gpurun_out/r04_close r04_close && ls profiles | grep r04_close
