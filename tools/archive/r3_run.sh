#!/bin/bash
# r03 GPU steps: each pytest run under its own time limit; stop at a crash / time limit
# (exit status >= 124), continue past ordinary test failures (status 1).
# usage: tools/r3_run.sh <out-dir> "<pytest args>" [timeout] ["<pytest args>" timeout] ...
set -u
out=$1; shift
mkdir -p "$out"
i=0
while [ $# -ge 2 ]; do
  args=$1; t=$2; shift 2; i=$((i + 1))
  echo "== step $i: pytest $args (limit ${t}s)"
  timeout -k 10 "$t" python -u -m pytest -x -v --timeout "$t" --timeout-method thread \
      -p no:cacheprovider $args > "$out/step$i.log" 2>&1
  rc=$?
  tail -5 "$out/step$i.log"
  if [ $rc -ge 124 ]; then echo "step $i ended with $rc: stopping"; exit $rc; fi
done
