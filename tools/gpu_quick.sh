#!/bin/bash
# Quick GPU pass: GPU tests (skip with NOTEST=1), then one bench line per
# "config:order" argument (LAYOUT=by_key for the layout study).
O=$GRAFT_REPO_ROOT/gpurun_out/quick
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log
  if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $O/tests.log | head; exit 1; fi
fi
for a in "$@"; do
  c=${a%%:*}; o=${a#*:}
  timeout -k 10 200 python -u bench.py --config $c --order $o ${LAYOUT:+--layout $LAYOUT} --steps 10 --warmup 3 --cpu-seconds 0 > $O/b_${c}_$o.json 2> $O/b.err || { echo "fail $a"; tail -3 $O/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_${c}_$o.json').read().strip().split(chr(10))[-1]); print('$a', d['value'], d['kernels_ms'], d.get('check'))"
done
