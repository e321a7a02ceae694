#!/bin/bash
# Round-2: register-transposed field backward — A/B diagnostic, parity tests, then the
# bench with each backward generation, then a rocprofv3 kernel trace of the default.
set -o pipefail
OUT=gpurun_out/${1:-r2s2b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/field_ab_diag.py > "$OUT/ab_diag.log" 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k "field" --timeout 300 --timeout-method thread > "$OUT/pytest_field.log" 2>&1 || exit $?
for m in rt lds rt; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --field-bwd $m > "$OUT/bench_$m.log" 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 10 --no-cpu-baseline --no-kernel-timer --spec-peaks > "$OUT/trace.log" 2>&1 || exit $?
echo done
