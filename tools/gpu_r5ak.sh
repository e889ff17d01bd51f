#!/bin/bash
# r5ak: mixed-suite backfill (QPP_COSCHED=1: ChaCha20 on a side stream forked before the 1024-thread GCM launch, its workgroups filling CUs as GCM workgroups leave)
# against sequential launches, config 5,
# interleaved; parity of the mixed tests under the switch first
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5ak; mkdir -p $O
QPP_COSCHED=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bucketing.py -k "config5 or planned_equals or ragged" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do
  for m in 0 1; do
    QPP_COSCHED=$m timeout -k 10 200 python -u bench.py --config 5 --steps 20 --warmup 5 --cpu-seconds 0 --cpu-all-cores 0 --no-e2e > $O/b_${m}_$rep.json 2> $O/b_${m}_$rep.err || { echo "fail $m"; tail -5 $O/b_${m}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${m}_$rep.json').read().strip().split(chr(10))[-1]); print('cosched=$m $rep', d['value'], d['kernels_ms'], d['status_ok'])"
  done
done
