#!/bin/bash
# Field forward uniform-tile form: bit-identity tests, then the probe A/B (general vs
# uniform-tile) and one bench run.
set -o pipefail
mkdir -p gpurun_out/r2s
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "field" > gpurun_out/r2s/tests.log 2>&1 || { tail -40 gpurun_out/r2s/tests.log; exit 1; }
tail -3 gpurun_out/r2s/tests.log
for m in 0 1 0 1; do
  echo "== fwd mode $m"
  timeout -k 10 120 python -u tools/field_probe.py --iters 10 --fwd-mode $m || exit $?
done
timeout -k 10 300 python -u bench.py > gpurun_out/r2s/bench.log 2>&1 || { tail -30 gpurun_out/r2s/bench.log; exit 1; }
tail -1 gpurun_out/r2s/bench.log | cut -c1-300
