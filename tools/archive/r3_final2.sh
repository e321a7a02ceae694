#!/bin/bash
# r03 closing run: the whole GPU suite (one process, thread timeouts), smoke(), the default
# bench line; then, given variants (baseline committed bf16), their rocprof passes.
# usage: tools/r3_final2.sh <out-dir> [variant ...]
set -o pipefail
OUT=${1:-gpurun_out/final2}; shift; mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench.json.log" 2>&1 || { tail -20 "$OUT/bench.json.log"; exit 1; }
tail -1 "$OUT/bench.json.log" | cut -c1-240
if [ $# -gt 0 ]; then tools/r3_final_prof.sh "$OUT" "$@" || exit $?; fi
