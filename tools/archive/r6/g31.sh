#!/bin/bash
# r6 final: rocprof kernel trace + PMC (FETCH / WRITE / ATOMIC) + SQ passes (TAG=r06_final)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r06_final bash tools/r6/prof_final.sh
bash tools/archive/r6/g29.sh
