#!/bin/bash
# A/B of library builds under variants/<name>/libquicpp.so (GPU box): bench config $CFG.
set -uo pipefail
cd $GRAFT_REPO_ROOT
for v in base "$@"; do
  if [ "$v" = base ]; then LP=""; else LP="$GRAFT_REPO_ROOT/variants/$v"; fi
  for rep in 1 2; do
    LD_LIBRARY_PATH=$LP timeout -k 10 120 python bench.py --config ${CFG:-2} --packets ${PKTS:-0} --steps 30 --warmup 3 --cpu-seconds 0 > gpurun_out/ab_$v.json 2>/dev/null || { echo "fail $v"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['value'], d['kernels_ms'], d['status_ok'])"
  done
done
