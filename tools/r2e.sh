set -o pipefail
O=gpurun_out/r2e; mkdir -p $O
export TMPDIR=/tmp
ANR_INGP_PSNR_OUT=$O/psnr_ingp.json ANR_PSNR_OUT=$O/psnr_nerf.json timeout -k 10 1100 python -u -m pytest tests -v -m gpu --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
echo done
