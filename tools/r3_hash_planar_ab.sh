set -o pipefail
OUT=gpurun_out/r4d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 180 python3 tools/hash_fwd_ab.py --views 90 --modes 0,p,0,p --iters 20 > $OUT/ab.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/hit -o run --output-format csv -- python3 tools/hash_fwd_ab.py --views 90 --modes 0,p --iters 3 > $OUT/hit.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/hash_fwd_ab.py --views 90 --modes 0,p --iters 3 > $OUT/fetch.log 2>&1 || exit $?
echo done
