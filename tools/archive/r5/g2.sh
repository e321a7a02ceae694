# hash bwd on the bench state: dump ref + build states, time skip modes, SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g2; mkdir -p $O
P=tools/r5/hash_bwd_state.py
timeout -k 10 300 python -u $P dump --numerics reference --out /tmp/hb_ref.pt > $O/dump_ref.log 2>&1 || { tail -20 $O/dump_ref.log; exit 1; }
tail -2 $O/dump_ref.log
timeout -k 10 300 python -u $P dump --numerics build --out /tmp/hb_build.pt > $O/dump_build.log 2>&1 || { tail -20 $O/dump_build.log; exit 1; }
tail -2 $O/dump_build.log
for st in ref build; do for k in 0 1 2; do
ANR_HASH_SKIP0=$k timeout -k 10 120 python -u $P time --state /tmp/hb_$st.pt > $O/time_${st}_$k.log 2>&1 || { tail -20 $O/time_${st}_$k.log; exit 1; }
echo "$st skip$k: $(grep median $O/time_${st}_$k.log | cut -c1-120)"
done; done
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU"
for st in ref build; do
timeout -s KILL 120 rocprofv3 --pmc $C -d $O/sq_$st -o run --output-format csv -- python3 $P time --state /tmp/hb_$st.pt --iters 3 > $O/sq_$st.log 2>&1 || { tail -20 $O/sq_$st.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum -d $O/tcc_ref -o run --output-format csv -- python3 $P time --state /tmp/hb_ref.pt --iters 3 > $O/tcc_ref.log 2>&1 || { tail -20 $O/tcc_ref.log; exit 1; }
rm -f /tmp/hb_ref.pt /tmp/hb_build.pt
echo done
