#!/bin/bash
# Round 6: D2H / H2D rates into hipHostMalloc'd memory over several processes,
# with the NUMA node of the pages and of the GPU.
set -uo pipefail
cd $GRAFT_REPO_ROOT
for f in 0 0 0 0 0 0; do
  timeout -k 5 60 ./tools/d2h_probe $f | grep -v "rep 1\|rep 0" || exit 1
done
numactl -H 2>/dev/null | head -3 || true
