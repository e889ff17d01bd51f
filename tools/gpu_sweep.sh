#!/bin/bash
# Bench every BASELINE config (+ the north-star 1Mi AES-128-GCM size) on one GPU.
set -uo pipefail
TAG=${1:-r1}
O=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
for c in 2 3 4 5; do
  timeout -k 10 200 python -u bench.py --config $c --cpu-seconds 3 > $O/sweep_${TAG}_c$c.json 2>$O/sweep_${TAG}_c$c.err || { echo "config $c failed"; tail $O/sweep_${TAG}_c$c.err; exit 1; }
  cat $O/sweep_${TAG}_c$c.json
done
timeout -k 10 200 python -u bench.py --config 2 --packets 1048576 --e2e --cpu-seconds 0 > $O/sweep_${TAG}_1mi.json 2>$O/sweep_${TAG}_1mi.err || { echo "1mi failed"; tail $O/sweep_${TAG}_1mi.err; exit 1; }
cat $O/sweep_${TAG}_1mi.json
