set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export ANR_INGP_PSNR_OUT=gpurun_out/r4_ingp_oracle_records.json
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "field" > gpurun_out/r4_field_test.log 2>&1 || { tail -40 gpurun_out/r4_field_test.log; exit 1; }
tail -2 gpurun_out/r4_field_test.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 850 --timeout-method thread tests/test_ingp_oracle_gpu.py > gpurun_out/r4_ingp_oracle.log 2>&1 || { tail -40 gpurun_out/r4_ingp_oracle.log; exit 1; }
tail -15 gpurun_out/r4_ingp_oracle.log
