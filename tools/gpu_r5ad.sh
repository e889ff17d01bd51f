#!/bin/bash
# r5ad: GCM persistent kernel with a launch-wide pool for the last 1/12 or
# 1/25 of the items (study build: device-global counters, one stream) against
# static shares; correctness pass, bench mode interleaved, then the probe's
# workgroup ends by XCD
set -uo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 5 60 tools/probe_pool12 1048576 0 | grep -E "status|diffs|bad" || exit 1
timeout -k 5 60 tools/probe_pool12 1048576 1 | grep -E "status|bad" || exit 1
for r in 1 2 3; do
  for v in base pool12 pool25; do
    for a in "1048576 0" "1048576 1" "65536 0"; do
      echo "$v $a $r $(timeout -k 5 60 tools/probe_$v $a bench)" || exit 1
    done
  done
done
timeout -k 5 60 tools/probe_pool12_prb 1048576 0 | grep -E "us \(event\)|wave ends|workgroup ends" || exit 1
