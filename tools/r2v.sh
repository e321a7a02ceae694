#!/bin/bash
# Historical (r02): the HASH_BWD_STATIC variant was removed after this run
# (profiles/r02_hash_bwd_static_count_failed.log).
# Hash-grid backward with a static count of vector-memory instructions per batch
# (HASH_BWD_STATIC=1: buffer atomics with out-of-range offsets for idle lanes, full
# batches in their own loop): A/B vs the product library, then the hash GPU tests.
set -o pipefail
for v in prod static prod static; do
  echo "== $v"
  if [ $v = prod ]; then unset ANR_HIP_LIB; else export ANR_HIP_LIB=$PWD/exp_libs/libanr_hb_$v.so; fi
  timeout -k 10 120 python -u tools/hash_bwd_ab.py --modes 0 --iters 10 2>&1 | grep -v amdgpu.ids || exit $?
done
export ANR_HIP_LIB=$PWD/exp_libs/libanr_hb_static.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "hash or ingp or step" 2>&1 | tail -3
