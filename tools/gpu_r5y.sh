#!/bin/bash
# r5y: progress priority for the last items of each GCM workgroup share
# (tail16 / tail24 / tail32: items of the share's last 16 / 24 / 32 with
# priority; 512-thread launches of <= 1 item per wave have every item in the
# tail) against the base engine; probe harness bench mode, interleaved
set -uo pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for v in base tail16 tail24 tail32; do
    for a in "65536 0" "1048576 0" "1048576 1"; do
      echo "$v $a $r $(timeout -k 5 60 tools/probe_$v $a bench)" || exit 1
    done
  done
done
