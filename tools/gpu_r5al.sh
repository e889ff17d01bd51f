#!/bin/bash
# r5al: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the final
# tree for every bench config
set -uo pipefail
cd $GRAFT_REPO_ROOT
for c in ns 2 3 4 5; do
  bash tools/gpu_traffic.sh tr_r5_$c $c || exit 1
done
cat gpurun_out/traffic.json
