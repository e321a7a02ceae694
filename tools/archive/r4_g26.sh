set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for nm in reference build; do
  timeout -k 10 400 python -u tools/liveness.py --steps 40 --numerics $nm > gpurun_out/r4_liveness_$nm.log 2>&1 || { tail -20 gpurun_out/r4_liveness_$nm.log; exit 1; }
  echo "== $nm"; grep "^step" gpurun_out/r4_liveness_$nm.log | awk 'NR<=12 || NR%4==0'
done
