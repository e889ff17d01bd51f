#!/bin/bash
# r5z: GPU tests of the tree with progress priority in 512-thread GCM
# launches, then bench.py A/B against HEAD's engine (variants/head):
# config 2 (64 Ki, the 512-thread shape) and the north star (1024, unchanged)
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_r5z.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests_r5z.log; exit 1; }
tail -1 $O/gpu_tests_r5z.log
REPS=3 bash tools/gpu_ab5.sh r5z_ab "2 ns" head
