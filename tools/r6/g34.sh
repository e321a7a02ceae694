#!/bin/bash
# r6 close: rocprof kernel trace + PMC + SQ passes of the committed library (TAG=r06_close)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r06_close bash tools/r6/prof_final.sh
