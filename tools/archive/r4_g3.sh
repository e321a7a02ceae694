# hash-bwd chunk-length sweep (ANR_HASH_KB) at the per-rank (1024 rays) and bench (8192) shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for R in 1024 8192; do
  for KB in 32 64 128 256 512 1024; do
    ANR_HASH_KB=$KB timeout -k 10 120 python -u tools/hash_bwd_ab.py --rays $R --modes 0 --iters 10 > gpurun_out/r4_ksweep_${R}_${KB}.log 2>&1 || exit 1
    echo "rays $R KB $KB: $(grep 'avg' gpurun_out/r4_ksweep_${R}_${KB}.log)"
  done
done
