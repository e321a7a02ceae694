set -o pipefail
# SQ counters of hash backward v2 (mode 0) and v3 (mode 8) on the bench coordinates
O=gpurun_out/r2p; mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS"
P2="SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d "$O/p$i" -o run --output-format csv -- python3 tools/hash_bwd_ab.py --modes 0,8 --iters 4 > "$O/p$i.log" 2>&1 || exit $?
done
python3 tools/pmc_table.py $O > $O/table.txt
echo done
