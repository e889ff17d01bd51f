#!/bin/bash
# GPU tests, then per-call latency of the object API (tools/bench_python_layer.py)
# for the in-tree library and for variants/<name> builds: tools/gpu_small.sh variant...
set -uo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_small.log 2>&1
  rc=$?; tail -1 gpurun_out/t_small.log
  if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/t_small.log | head -20; exit 1; fi
fi
for v in base "$@"; do
  if [ "$v" = base ]; then LP=""; else LP="$GRAFT_REPO_ROOT/variants/$v"; fi
  LD_LIBRARY_PATH=$LP timeout -k 10 200 python tools/bench_python_layer.py --reps ${REPS:-500} > gpurun_out/pl_$v.json 2> gpurun_out/pl_$v.err || { echo "fail $v"; tail -5 gpurun_out/pl_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/pl_$v.json')); print('$v', d['latency_us'])"
done
