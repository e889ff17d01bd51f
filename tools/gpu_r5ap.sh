#!/bin/bash
# r5ap: pool share 1/12 (tree) against 1/6 and 1/24 (variants), north star
set -uo pipefail
cd $GRAFT_REPO_ROOT
REPS=4 bash tools/gpu_ab5.sh r5ap_ab "ns" div6 div24
