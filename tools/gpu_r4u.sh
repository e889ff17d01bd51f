#!/bin/bash
# r4u: same-box A/B of variants/$2 against the tree at config 3 (64 Ki and 1 Mi).
set -uo pipefail
TAG=${1:-r4u}; V=${2:-wpe5}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
for p in 0 1048576 0; do
  CFG=3 PKTS=$p bash tools/ab_lib.sh $V > $O/ab_c3_$p.txt 2>&1 || { echo "ab $p failed"; cat $O/ab_c3_$p.txt; exit 1; }
  echo "== config 3 packets $p"; cat $O/ab_c3_$p.txt
done
