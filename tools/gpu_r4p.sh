#!/bin/bash
# r4p: GPU tests, object-API latency, and the lone/quad sweep with the
# default per-suite thresholds against QPP_LONE=0.
set -uo pipefail
TAG=${1:-r4p}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python tools/lat_probe.py > $O/lat_probe.txt 2>&1 || { echo "lat_probe failed"; cat $O/lat_probe.txt; exit 1; }
cat $O/lat_probe.txt
export LONE_SIZES=1,16,256,4096,8192,16384
timeout -k 10 300 python tools/lone_sizes.py > $O/default.jsonl 2> $O/default.err || { echo "sweep failed"; tail -20 $O/default.err; exit 1; }
QPP_LONE=0 timeout -k 10 300 python tools/lone_sizes.py > $O/quad.jsonl 2> $O/quad.err || { echo "quad sweep failed"; tail -20 $O/quad.err; exit 1; }
cat $O/default.jsonl $O/quad.jsonl
