#!/bin/bash
# SQ counter passes for the hash-grid forward (v6) and backward (v2) at bench size
# (tools/hash_fwd_ab.py / tools/hash_bwd_ab.py, bench coordinates), one rocprofv3 run
# per counter set. usage: tools/r3_hash_pmc.sh <out-dir>
set -o pipefail
OUT=${1:-gpurun_out/hash_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_INSTS_SALU,SQ_INSTS_VALU"
P2="SQ_INSTS_VMEM,SQ_ACTIVE_INST_VMEM,SQ_ACTIVE_INST_MISC,SQ_INSTS_BRANCH,SQ_BUSY_CYCLES,SQ_INST_CYCLES_SALU,SQ_WAIT_INST_LDS,SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc ${P//,/ } -d "$OUT/fwd_p$i" -o run --output-format csv -- \
    python3 tools/hash_fwd_ab.py --modes 0 --iters 3 > "$OUT/fwd_p$i.log" 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc ${P//,/ } -d "$OUT/bwd_p$i" -o run --output-format csv -- \
    python3 tools/hash_bwd_ab.py --modes 0 --iters 3 > "$OUT/bwd_p$i.log" 2>&1 || exit $?
done
echo done
