set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d gpurun_out/r4_atomic_probe -o run --output-format csv -- python3 tools/atomic_model_probe.py > gpurun_out/r4_atomic_probe.log 2>&1 || { tail -20 gpurun_out/r4_atomic_probe.log; exit 1; }
grep "instrument" gpurun_out/r4_atomic_probe.log
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r4_atomic_probe/**/*counter_collection.csv", recursive=True):
    rows = [r for r in csv.DictReader(open(f)) if "hashgrid_bwd_v2" in r["Kernel_Name"]]
    for r in rows:
        print(r.get("Dispatch_Id"), r["Kernel_Name"][:60], r["Counter_Value"])
PY
