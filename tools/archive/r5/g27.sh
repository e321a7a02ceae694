#!/bin/bash
# r5: cold-start liveness at batch 1,024 (both numerics, beside the oracle's), the
# cold-start headline number, and SQ counters of the current NeRF kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g27; mkdir -p $O
for n in reference build; do
timeout -k 10 300 python -u tools/liveness.py --numerics $n --batch 1024 --steps 30 > $O/live_$n.log 2>&1 || { tail -20 $O/live_$n.log; exit 1; }
echo "== $n"; grep step $O/live_$n.log | cut -c1-100
done
timeout -k 10 300 python -u bench.py --cold-start --no-alt-numerics --no-cpu-baseline > $O/bench_cold.json.log 2>&1 || { tail -30 $O/bench_cold.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench_cold.json.log cold_start
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- python3 tools/r5/nerf_gemm_probe.py 256x256 > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
python3 - <<'PY' > $O/nerf_sq.txt
import csv, glob, collections
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/r5_g27/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    if "nerfmlp" not in k and "Cijk" not in k:
        continue
    med = {c: sorted(v)[len(v) // 2] for c, v in d.items()}
    print("==", k)
    for c in sorted(med):
        print(f"  {c:28s} {med[c]:.4g}")
PY
rm -rf $O/p1 $O/p2
cat $O/nerf_sq.txt | head -60
