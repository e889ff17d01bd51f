#!/bin/bash
# r5ag: bench.py A/B, single-key pool against HEAD's engine: north star, config 4
set -uo pipefail
cd $GRAFT_REPO_ROOT
REPS=4 bash tools/gpu_ab5.sh r5ag_ab "ns 4" head
