#!/bin/bash
# Layout study: the batch shifted by QPP_BENCH_SHIFT bytes in its buffers
# (5: every payload on a 16-byte boundary), north star and config 3.
set -uo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/shift
for rep in 1 2; do
  for cfg in ns 3; do
    for sh in 0 5; do
      QPP_BENCH_SHIFT=$sh timeout -k 10 150 python -u bench.py --config $cfg --steps 20 --warmup 5 --cpu-seconds 0 --cpu-all-cores 0 > gpurun_out/shift/b_${cfg}_$sh.json 2> gpurun_out/shift/b.err || { echo "fail $cfg $sh"; tail -3 gpurun_out/shift/b.err; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/shift/b_${cfg}_$sh.json').read().strip().split(chr(10))[-1]); print('$cfg shift=$sh', d['value'], d['kernels_ms'], d['status_ok'])"
    done
  done
done
