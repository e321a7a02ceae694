set -o pipefail
# hash forward v6: parity (all hash tests incl. the v6 mode), then bench A/B of mode 0 vs 6
O=gpurun_out/r2k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k "hashgrid" --timeout 300 --timeout-method thread > $O/pytest_hash.log 2>&1 || exit $?
for m in 0 6 0 6; do
  ANR_HASHGRID_MODE=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline --spec-peaks > $O/bench_mode$m.log 2>&1 || exit $?
  grep -h metric $O/bench_mode$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('mode $m', d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items() if k.startswith('hash')})" >> $O/summary.txt
done
echo done
