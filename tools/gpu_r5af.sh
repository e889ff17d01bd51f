#!/bin/bash
# r5af: pool for single-key launches only -- the pool test and the parity
# files, then bench.py A/B against HEAD's engine, north star and config 4
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_parity.py tests/test_gpu_bucketing.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_r5af.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests_r5af.log; exit 1; }
tail -1 $O/gpu_tests_r5af.log
REPS=4 bash tools/gpu_ab5.sh r5af_ab "ns 4" head
