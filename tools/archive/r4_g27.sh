set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/liveness.py --steps 40 --numerics reference --switch-at 10 > gpurun_out/r4_liveness_switch.log 2>&1 || { tail -20 gpurun_out/r4_liveness_switch.log; exit 1; }
grep "^step\|^--" gpurun_out/r4_liveness_switch.log | awk 'NR<=16 || NR%3==0'
