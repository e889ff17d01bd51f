#!/bin/bash
# r5ao: the GCM item pool on and off (QPP_GCM_POOL=0), north star, bench.py,
# interleaved, 4 reps (another box for the pool's box-dependent gain)
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5ao}; mkdir -p $O
for r in 1 2 3 4; do
  for m in 1 0; do
    QPP_GCM_POOL=$m timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --cpu-seconds 0 --cpu-all-cores 0 --no-e2e > $O/b_${m}_$r.json 2> $O/b_${m}_$r.err || { echo "fail $m"; tail -5 $O/b_${m}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${m}_$r.json').read().strip().split(chr(10))[-1]); print('pool=$m $r', d['value'], d['kernels_ms'])"
  done
done
