#!/bin/bash
# A/B of engine variants as standalone probe binaries (GPU box, no Python).
#   SUITES="0 1" PKTS=65536 tools/ab_probe.sh base f2:QPP_WG_GCM=768 ...
# Each spec is a tools/probe_<name> binary plus optional env (comma separated).
# First a correctness pass per spec (status histogram, round-trip diffs), then
# two interleaved timing passes.
set -uo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # spec suite mode
  local spec=$1 s=$2 mode=$3 name=${1%%:*} envs=""
  [[ $spec == *:* ]] && envs=${spec#*:}
  env ${envs//,/ } timeout -k 5 60 tools/probe_$name ${PKTS:-65536} $s $mode
}
for s in ${SUITES:-0}; do
  for spec in "$@"; do
    run $spec $s check > gpurun_out/abchk_${spec//[:=,]/_}_$s.log 2>&1 || { echo "FAIL check $spec suite $s"; exit 1; }
    grep -E "bad|diffs" gpurun_out/abchk_${spec//[:=,]/_}_$s.log | tr '\n' ' ' | sed "s/^/check $spec suite $s: /"; echo
  done
done
for rep in 1 2; do
  for s in ${SUITES:-0}; do
    for spec in "$@"; do
      printf '%-24s suite %s: ' "$spec" $s
      run $spec $s bench || { echo "FAIL $spec"; exit 1; }
    done
  done
done
