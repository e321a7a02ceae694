# hash bwd: batch coordinates through scalar loads (new), + dL/dy loads paired over b lanes
# (gpair); hash tests on both, then bench A/B/C (base = HEAD .so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k hash > gpurun_out/r4_g38_test.log 2>&1 || { tail -40 gpurun_out/r4_g38_test.log; exit 1; }
tail -1 gpurun_out/r4_g38_test.log
ANR_HIP_LIB=$PWD/abso/libanr_hip_gpair.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k hash > gpurun_out/r4_g38_test_gpair.log 2>&1 || { tail -40 gpurun_out/r4_g38_test_gpair.log; exit 1; }
tail -1 gpurun_out/r4_g38_test_gpair.log
for rep in 1 2; do
for v in base new gpair; do
case $v in base) export ANR_HIP_LIB=$PWD/abso/libanr_hip_base.so;; gpair) export ANR_HIP_LIB=$PWD/abso/libanr_hip_gpair.so;; *) unset ANR_HIP_LIB;; esac
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r4_g38_${v}_$rep.json.log 2>&1 || exit 1
python3 - $v $rep <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/r4_g38_{sys.argv[1]}_{sys.argv[2]}.json.log") if x.startswith("{")][-1]
d = json.loads(l); r = d["roofline"]; a = d["alt_numerics"]
print(sys.argv[1], "ref", d["value"], d["ms_per_step"], "| build", a["ms_per_step"], "| hash_bwd live", r["avg_ms"], r["frac"], r.get("atomic_requests_before_after"), "| field_bwd", d["kernels"]["field_bwd"]["avg_ms"], "hash_bwd", d["kernels"]["hash_bwd"]["avg_ms"])
PY
done
done
