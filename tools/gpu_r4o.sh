#!/bin/bash
# r4o: lone / quad crossover sweep (tools/lone_sizes.py).
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4o}; mkdir -p $O
export LONE_SIZES=${LONE_SIZES:-1,4,16,64,256,1024,4096}
for m in lone quad; do
  if [ $m = lone ]; then E="QPP_LONE_MAX=1048576"; else E="QPP_LONE=0"; fi
  env $E timeout -k 10 300 python tools/lone_sizes.py > $O/$m.jsonl 2> $O/$m.err || { echo "$m sweep failed"; tail -20 $O/$m.err; exit 1; }
done
cat $O/lone.jsonl $O/quad.jsonl
