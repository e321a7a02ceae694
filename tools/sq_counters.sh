#!/bin/bash
# SQ counter pass (rocprofv3 --pmc, kernel trace only) over the hash and field probes:
# where wave cycles go (issuing / parked on s_waitcnt / issue-stalled) and the instruction
# mix per kernel. Usage: tools/sq_counters.sh [outdir]
set -o pipefail
OUT=${1:-gpurun_out/sq}
mkdir -p "$OUT"
export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS"
for probe in hash field; do
  timeout -k 10 300 rocprofv3 --pmc $C1 -d "$OUT/$probe" -o run --output-format csv -- python3 tools/${probe}_probe.py > "$OUT/$probe.log" 2>&1 || exit $?
done
echo done
