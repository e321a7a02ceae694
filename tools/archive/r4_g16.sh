set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/r4_g15.sh && bash tools/r4_g14.sh
