#!/bin/bash
# Round-4 pooled two-workgroup GCM pass: GPU tests, then same-box interleaved
# A/B against the round-3 kernel (variants/r3base) at the north star and
# configs 2, 4, 5.
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_r4e.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests_r4e.log; exit 1; }
tail -1 $O/gpu_tests_r4e.log
for c in ns 2 4 5; do
  CFG=$c bash tools/ab_lib.sh r3base > $O/ab_r4e_c$c.txt 2>&1 || { echo "ab $c failed"; cat $O/ab_r4e_c$c.txt; exit 1; }
  echo "== config $c"; cat $O/ab_r4e_c$c.txt
done
