# SQ counters of the ref16 composite kernels (tools/ref16_bench.py) at R = 1 and 2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS"
for R in 1 2; do
  ANR_REF16_R=$R timeout -s KILL 120 rocprofv3 --pmc $C1 -d gpurun_out/r4_sq16_$R -o run --output-format csv -- python3 tools/ref16_bench.py --iters 4 > gpurun_out/r4_sq16_$R.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for R in (1, 2):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/r4_sq16_{R}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "ref16" not in k: continue
            kk = "fwd" if "fwd_kernel" in k else ("bwd" if "bwd_kernel" in k else k[:40])
            vals[kk][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for kk, d in vals.items():
        med = {c: sorted(v)[len(v) // 2] for c, v in d.items()}
        print(f"R={R} {kk}:", {c: f"{v:.4g}" for c, v in sorted(med.items())})
PY
