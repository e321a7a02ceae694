# hash bwd: skip zero-sum corners in cell-move flushes (ANR_HASH_SKIP0), alternating A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "hash" > gpurun_out/r4_g23_test.log 2>&1 || { tail -30 gpurun_out/r4_g23_test.log; exit 1; }
tail -1 gpurun_out/r4_g23_test.log
for rep in 1 2; do
  for S in 0 1; do
    ANR_HASH_SKIP0=$S timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4_skip0_${S}_${rep}.json.log 2>&1 || exit 1
    python3 - $S $rep <<'PY'
import json, sys
S, rep = sys.argv[1:]
l = [x for x in open(f"gpurun_out/r4_skip0_{S}_{rep}.json.log") if x.startswith("{")][-1]
d = json.loads(l); a = d["alt_numerics"]
print(f"skip0={S} rep={rep} ref {d['ms_per_step']} hash_bwd {d['kernels']['hash_bwd']['avg_ms']} live {d['roofline']['avg_ms']} | build {a['ms_per_step']} hash_bwd {a['kernels']['hash_bwd']['avg_ms']}")
PY
  done
done
