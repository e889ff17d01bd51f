#!/bin/bash
# GCM blocks-per-lane study: GPU parity under QPP_GCM_BPL=2, then A/B bench
# lines (ns = north star; 4 = AES-256, 4096 keys) for BPL 1/2 and workgroup sizes.
set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/bpl
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ -z "${NOTEST:-}" ]; then
  QPP_GCM_BPL=2 timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_bpl2.log 2>&1
  rc=$?; tail -2 $O/tests_bpl2.log
  if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests_bpl2.log | head -20; exit 1; fi
fi
for cfg in ${CFGS:-ns 4}; do
  for v in ${VARS:-1:1024 2:1024 2:768 1:1024 2:1024}; do
    b=${v%%:*}; w=${v#*:}
    QPP_GCM_BPL=$b QPP_WG_GCM=$w timeout -k 10 150 python -u bench.py --config $cfg --steps 20 --warmup 5 --cpu-seconds 0 > $O/b_${cfg}_${b}_${w}.json 2> $O/b.err || { echo "fail $cfg $v"; tail -3 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${cfg}_${b}_${w}.json').read().strip().split(chr(10))[-1]); print('$cfg bpl=$b wg=$w', d['value'], d['kernels_ms'], d.get('check'))"
  done
done
