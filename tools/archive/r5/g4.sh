set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_g4; mkdir -p $O
for m in 0 1 2; do
ANR_HASH_PLANE_MAP=$m timeout -k 10 120 python -u tools/r5/hash_fwd_planes_probe.py > $O/planes_$m.log 2>&1 || { tail -20 $O/planes_$m.log; exit 1; }
tail -1 $O/planes_$m.log
done
timeout -k 10 1000 python -u tools/r5/grad_arms_diag.py --out gpurun_out/r5_grad_arms.json > gpurun_out/r5_grad_arms.log 2>&1 || { tail -20 gpurun_out/r5_grad_arms.log; exit 1; }
echo done
