#!/bin/bash
# Same-box interleaved A/B of the current tree against variants/r3base at the
# north star and configs 2, 4, 5 (tools/ab_lib.sh).
set -uo pipefail
cd $GRAFT_REPO_ROOT
for c in ns 2 4 5; do
  CFG=$c bash tools/ab_lib.sh ${2:-r3base} > gpurun_out/ab_${1:-r4f}_c$c.txt 2>&1 || { echo "ab $c failed"; cat gpurun_out/ab_${1:-r4f}_c$c.txt; exit 1; }
  echo "== config $c"; cat gpurun_out/ab_${1:-r4f}_c$c.txt
done
