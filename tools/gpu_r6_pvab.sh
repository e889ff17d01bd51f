#!/bin/bash
# Round 6: interleaved A/B of bench-mode probe binaries (tools/pv_<name>, built
# by tools/build_probe_variants.sh) on one box:
#   gpurun -- bash tools/gpu_r6_pvab.sh TAG "packets suite" "variants..." [reps]
set -uo pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; SIZES=$2; VARS=$3; REPS=${4:-3}
O=gpurun_out/$TAG; mkdir -p $O
for rep in $(seq 1 $REPS); do
  for sz in $SIZES; do
    n=${sz%:*}; su=${sz#*:}
    for v in $VARS; do
      r=$(timeout -k 5 60 ./tools/pv_$v $n $su bench 2>&1) || { echo "fail $v $n $su: $r"; exit 1; }
      echo "$v $n $su $rep $r" | tee -a $O/ab.txt
    done
  done
done
