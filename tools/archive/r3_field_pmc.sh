#!/bin/bash
# Field backward generations 1 (MFMA transposes) and 2 (LDS transposes): timing, then SQ
# PMC passes (one rocprofv3 run per counter set and mode).
# usage: tools/r3_field_pmc.sh <out-dir>
set -o pipefail
OUT=${1:-gpurun_out/field_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in 1 2; do
  timeout -k 10 120 python3 tools/field_bwd_pmc.py --mode $m --iters 20 >> "$OUT/times.log" 2>&1 || exit $?
done
P1="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_MISC,SQ_ACTIVE_INST_SCA,SQ_INSTS_SALU,SQ_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  for m in 1 2; do
    timeout -s KILL 90 rocprofv3 --pmc ${P//,/ } -d "$OUT/p${i}_m$m" -o run --output-format csv -- \
      python3 tools/field_bwd_pmc.py --mode $m --iters 3 > "$OUT/p${i}_m$m.log" 2>&1 || exit $?
  done
done
echo done
