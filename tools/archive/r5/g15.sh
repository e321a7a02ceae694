#!/bin/bash
# r5: SQ counters of the NeRF dense-layer kernels and hipBLASLt's on the 256x256 shape
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g15; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- python3 tools/r5/nerf_gemm_probe.py 256x256 > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/r5_g15/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:70]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    if "nerfmlp" not in k and "Cijk" not in k:
        continue
    med = {c: sorted(v)[len(v) // 2] for c, v in d.items()}
    print("==", k)
    for c in sorted(med):
        print(f"  {c:28s} {med[c]:.4g}")
    wc = med.get("SQ_WAVE_CYCLES")
    bc = med.get("SQ_BUSY_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in med:
                print(f"  {c + '/WAVE':28s} {med[c] / wc:.3f}")
PY
