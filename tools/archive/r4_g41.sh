# SQ / TA / TCP counters of the bench step (reference numerics, warm start) on the final
# tree: the hash bwd walk after the scalar coordinate loads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BENCH_ARGS="--no-alt-numerics" bash tools/sq_bench.sh gpurun_out/r04_sq_close || exit 1
python3 tools/pmc_table.py gpurun_out/r04_sq_close > gpurun_out/r04_sq_close.md 2>&1 || { tail gpurun_out/r04_sq_close.md; exit 1; }
cat gpurun_out/r04_sq_close.md
