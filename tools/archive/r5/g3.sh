# bench JSON smoke with the r05 fields + settle study (warmup sweep) + liveness trajectory
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graph_gpu.py > $O/test_graph.log 2>&1 || { tail -40 $O/test_graph.log; exit 1; }
tail -1 $O/test_graph.log
timeout -k 10 400 python -u bench.py > $O/bench_default.json.log 2>&1 || { tail -30 $O/bench_default.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench_default.json.log default
for w in 100 300; do
timeout -k 10 400 python -u bench.py --warmup $w --no-cpu-baseline --no-alt-numerics > $O/bench_w$w.json.log 2>&1 || { tail -30 $O/bench_w$w.json.log; exit 1; }
python3 tools/r5/bench_line.py $O/bench_w$w.json.log warmup$w
done
timeout -k 10 400 python -u tools/liveness.py --steps 400 --switch-at 10 --numerics reference > $O/liveness_ref400.log 2>&1 || { tail -30 $O/liveness_ref400.log; exit 1; }
awk 'NR%20==1' $O/liveness_ref400.log | cut -c1-150
