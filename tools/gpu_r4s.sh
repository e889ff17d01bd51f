#!/bin/bash
# r4s: same-box A/B of variants/$2 against the tree at the north star,
# configs 2 and 4, and the north star again (tools/ab_lib.sh, interleaved).
set -uo pipefail
TAG=${1:-r4s}; V=${2:-andor}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
for c in ns 2 4 ns; do
  CFG=$c bash tools/ab_lib.sh $V > $O/ab_c$c.txt 2>&1 || { echo "ab $c failed"; cat $O/ab_c$c.txt; exit 1; }
  echo "== config $c"; cat $O/ab_c$c.txt
done
