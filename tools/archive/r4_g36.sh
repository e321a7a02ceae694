# final tree: full GPU suite and smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/r4_gpu_suite_final.log 2>&1 || { tail -40 gpurun_out/r4_gpu_suite_final.log; exit 1; }
tail -2 gpurun_out/r4_gpu_suite_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke_final.log 2>&1 || { tail -20 gpurun_out/r4_smoke_final.log; exit 1; }
tail -2 gpurun_out/r4_smoke_final.log
