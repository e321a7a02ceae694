set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g5; mkdir -p $O
timeout -k 10 120 python -u tools/r5/mfma_precision.py > $O/mfma_precision.log 2>&1 || { tail -20 $O/mfma_precision.log; exit 1; }
cat $O/mfma_precision.log
for mode in 0 9; do
ANR_HASHGRID_MODE=$mode timeout -k 10 120 python -u tools/r5/hash_fwd_planes_probe.py > $O/planes_mode$mode.log 2>&1 || { tail -20 $O/planes_mode$mode.log; exit 1; }
echo "mode $mode: $(tail -1 $O/planes_mode$mode.log)"
done
