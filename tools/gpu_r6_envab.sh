#!/bin/bash
# Round 6: interleaved A/B of one bench-mode probe binary (tools/pv_base) under
# environment switches, on one box:
#   gpurun -- bash tools/gpu_r6_envab.sh TAG "packets:suite ..." "name=ENV=VAL ..." [reps]
set -uo pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; SIZES=$2; VARS=$3; REPS=${4:-3}
O=gpurun_out/$TAG; mkdir -p $O
for rep in $(seq 1 $REPS); do
  for sz in $SIZES; do
    n=${sz%:*}; su=${sz#*:}
    for v in $VARS; do
      name=${v%%=*}; kv=${v#*=}
      r=$(env $kv timeout -k 5 60 ./tools/pv_base $n $su bench 2>&1) || { echo "fail $v $n $su: $r"; exit 1; }
      echo "$name $n $su $rep $r" | tee -a $O/ab.txt
    done
  done
done
