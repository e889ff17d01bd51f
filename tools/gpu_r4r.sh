#!/bin/bash
# r4r: GPU tests, then object-API latency with the kernel staging its call
# (default) and with QPP_LONE_STAGE=0 (one copy), same box, interleaved.
set -uo pipefail
TAG=${1:-r4r}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for rep in 1 2; do
  for st in 1 0; do
    QPP_LONE_STAGE=$st timeout -k 10 120 python tools/lat_probe.py > $O/lat_stage${st}_$rep.txt 2>&1 || { echo "lat_probe failed"; cat $O/lat_stage${st}_$rep.txt; exit 1; }
    echo "== QPP_LONE_STAGE=$st rep $rep"; grep us $O/lat_stage${st}_$rep.txt
  done
done
timeout -k 10 300 python tools/bench_python_layer.py --packets 16384 > $O/python_layer.json 2> $O/python_layer.err || { echo "python layer failed"; tail -20 $O/python_layer.err; exit 1; }
cat $O/python_layer.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o lat -- python3 tools/lat_trace.py 2000 > $O/lat_trace.log 2>&1 || { echo "trace failed"; tail -20 $O/lat_trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cat {} \;
