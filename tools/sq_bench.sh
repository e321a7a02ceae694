#!/bin/bash
# SQ / TA / TCP counter passes over the bench step in steady state (12 warm-up steps):
# where each hot kernel's wave cycles go and its instruction mix. One pass per counter
# group (gfx950 slot limits: 8 SQ, 2 TA, 4 TCP, 2 GRBM per pass).
# Usage: tools/sq_bench.sh [outdir]; summarise with tools/pmc_table.py <outdir>
set -o pipefail
OUT=${1:-gpurun_out/sq_bench}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 12 --no-cpu-baseline --no-kernel-timer --spec-peaks ${BENCH_ARGS}"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS"
P2="SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
P3="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P -d "$OUT/p$i" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1 || exit $?
done
echo done
