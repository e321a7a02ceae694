#!/bin/bash
# r03 final rocprofv3 passes (tools/prof.sh) for the bench line's variants.
# usage: tools/r3_final_prof.sh <out-dir> <variant...>   (baseline | committed | bf16)
set -o pipefail
OUT=$1; shift
for v in "$@"; do
  case $v in
    baseline) BENCH_ARGS="" tools/prof.sh "$OUT/prof" || exit $? ;;
    committed) BENCH_ARGS="--variant committed" tools/prof.sh "$OUT/prof_committed" || exit $? ;;
    bf16) BENCH_ARGS="--dtype bf16" tools/prof.sh "$OUT/prof_bf16" || exit $? ;;
  esac
done
echo done
