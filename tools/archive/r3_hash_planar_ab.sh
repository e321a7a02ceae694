#!/bin/bash
# r03 A/B of the XCD-affine level-pair forward (v8, anr_hashgrid_fwd_planar) against v6,
# with TCC hit/miss and FETCH_SIZE passes (profiles/r03_hash_levels.md §3). v8 was removed
# from the library after this measurement; the script needs commit be2df58's library.
set -o pipefail
OUT=gpurun_out/r4d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 180 python3 tools/hash_fwd_ab.py --views 90 --modes 0,p,0,p --iters 20 > $OUT/ab.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/hit -o run --output-format csv -- python3 tools/hash_fwd_ab.py --views 90 --modes 0,p --iters 3 > $OUT/hit.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/hash_fwd_ab.py --views 90 --modes 0,p --iters 3 > $OUT/fetch.log 2>&1 || exit $?
echo done
