#!/bin/bash
# Historical (r02): the --bwd-mode probe option and the uniform-tile backward it selected
# were reverted after this run (profiles/r02_field_bwd_uniform_tile_failed.log).
# Field backward uniform-tile form (scalar per-half directions): field GPU tests, probe
# A/B of anr_ingp_field_force_bwd 2 (general rt) vs 1 (uniform-tile rt), one bench run.
set -o pipefail
mkdir -p gpurun_out/r2t
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "field" > gpurun_out/r2t/tests.log 2>&1 || { tail -40 gpurun_out/r2t/tests.log; exit 1; }
tail -3 gpurun_out/r2t/tests.log
for m in 2 1 2 1; do
  echo "== bwd mode $m"
  timeout -k 10 120 python -u tools/field_probe.py --iters 10 --bwd-mode $m || exit $?
done
timeout -k 10 300 python -u bench.py > gpurun_out/r2t/bench.log 2>&1 || { tail -30 gpurun_out/r2t/bench.log; exit 1; }
tail -1 gpurun_out/r2t/bench.log | cut -c1-300
