#!/bin/bash
# r03: hash backward x-carry (mode 8) against the v2 default (mode 0): hash-grid parity
# tests, HIP-event A/B at bench size, memory-side atomic requests per launch (PMC).
# (Record of a removed experiment: mode 8 left the library after this run; profiles/r03_hash_bwd_xcarry_ab.log.)
set -o pipefail
OUT=${1:-gpurun_out/xc}; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k hashgrid -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest_hash.log" 2>&1 || { tail -30 "$OUT/pytest_hash.log"; exit 1; }
tail -1 "$OUT/pytest_hash.log"
timeout -k 10 300 python -u tools/hash_bwd_ab.py --modes 0,8,0,8 --iters 20 > "$OUT/ab.log" 2>&1 || exit $?
cat "$OUT/ab.log"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d "$OUT/atomic" -o run --output-format csv -- python3 tools/hash_bwd_ab.py --modes 0,8 --iters 2 > "$OUT/atomic.log" 2>&1 || exit $?
python3 - "$OUT/atomic" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(list)
for row in csv.DictReader(open(f[0])):
    if "hashgrid_bwd" in row["Kernel_Name"]:
        acc[row["Kernel_Name"][:90]].append(float(row["Counter_Value"]))
for k, v in acc.items():
    print(f"{k}: {len(v)} launches, mean {sum(v)/len(v):.4e} atomic requests")
PY
