#!/bin/bash
# r5ae: the launch-wide GCM item pool (key-table pool slots) -- GPU tests,
# then bench.py A/B against HEAD's engine (variants/head) on every config
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_r5ae.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests_r5ae.log; exit 1; }
tail -1 $O/gpu_tests_r5ae.log
REPS=3 bash tools/gpu_ab5.sh r5ae_ab "ns 4 5" head
