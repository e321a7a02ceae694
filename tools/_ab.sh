set -o pipefail
mkdir -p gpurun_out/ab
A="--steps 10 --warmup 3 --no-cpu-baseline --profile-steps 1"
timeout -k 10 200 python -u bench.py $A > gpurun_out/ab/default.log 2>&1 || exit $?
ANR_MLP_BWD_MIN_TILES=1 timeout -k 10 200 python -u bench.py $A > gpurun_out/ab/mintiles1.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py $A --no-fused-zero > gpurun_out/ab/nofz.log 2>&1 || exit $?
ANR_MLP_BWD_MIN_TILES=1 timeout -k 10 200 python -u bench.py $A --no-fused-zero > gpurun_out/ab/both.log 2>&1 || exit $?
echo done
