#!/bin/bash
# r5aj: chunked pool (QPP_POOL_CHUNK: chunks of 16 consecutive pooled items per
# workgroup, every 1024-thread launch incl. bucketed many-key ones) against the
# tree (per-item pool, single-key launches only); parity of the bucketed
# tests under the variant first
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/variants/chunk timeout -k 10 600 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_bucketing.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_r5aj.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests_r5aj.log; exit 1; }
tail -1 $O/gpu_tests_r5aj.log
REPS=3 bash tools/gpu_ab5.sh r5aj_ab "ns 4 5" chunk
