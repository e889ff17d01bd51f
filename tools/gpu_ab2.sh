#!/bin/bash
# GPU tests, then an A/B of the in-tree library against variants/<name>/
# builds on bench configs (one line per run): tools/gpu_ab2.sh tag cfg... -- variant...
set -uo pipefail
TAG=$1; shift
CFGS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do CFGS+=("$1"); shift; done
[ $# -gt 0 ] && shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log
  if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; fi
fi
for c in "${CFGS[@]}"; do
  for v in base "$@"; do
    if [ "$v" = base ]; then LP=""; else LP="$GRAFT_REPO_ROOT/variants/$v"; fi
    LD_LIBRARY_PATH=$LP timeout -k 10 150 python -u bench.py --config $c --packets ${PKTS:-0} --steps ${STEPS:-20} --warmup 5 --cpu-seconds 0 --cpu-all-cores 0 > $O/b_${c}_$v.json 2> $O/b_${c}_$v.err || { echo "fail $c $v"; tail -5 $O/b_${c}_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${c}_$v.json').read().strip().split(chr(10))[-1]); print('$c $v', d['value'], d['kernels_ms'], d.get('check'), d['status_ok'])"
  done
done
