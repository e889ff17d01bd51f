#!/bin/bash
# Round 6: phase probe of the packet kernels (tools/probe.hip, QPP_PROBE build):
#   gpurun -- bash tools/gpu_r6b_probe.sh TAG "packets suite" ...
set -uo pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for a in "$@"; do
  timeout -k 10 60 ./tools/probe $a > "$O/probe_${a// /_}.txt" 2>&1 || { echo "probe $a failed"; tail "$O/probe_${a// /_}.txt"; exit 1; }
  grep -A14 "^protect: waves" "$O/probe_${a// /_}.txt"
done
