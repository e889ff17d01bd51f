#!/bin/bash
# Round-3 final pass: tests, smoke, default bench, rehearsal, rocprof kernel
# trace (gpu_r3.sh), HBM traffic of the north star (FETCH_SIZE / WRITE_SIZE
# passes), then every config and the end-to-end line (gpu_sweep.sh).
set -uo pipefail
TAG=${1:-r3y}
cd $GRAFT_REPO_ROOT
bash tools/gpu_r3.sh $TAG || exit 1
bash tools/gpu_traffic.sh tr_$TAG ns || exit 1
bash tools/gpu_sweep.sh $TAG || exit 1
echo final-done $TAG
