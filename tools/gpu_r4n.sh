#!/bin/bash
# r4n: GPU tests, then the object-API latency with the lone kernels staging
# their call themselves and signalling completion through a pinned word.
#   gpurun -- bash tools/gpu_r4n.sh TAG
set -uo pipefail
TAG=${1:-r4n}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python tools/lat_probe.py > $O/lat_probe.txt 2>&1 || { echo "lat_probe failed"; cat $O/lat_probe.txt; exit 1; }
cat $O/lat_probe.txt
QPP_ZERO_COPY=0 timeout -k 10 120 python tools/lat_probe.py > $O/lat_probe_copies.txt 2>&1 || { echo "lat_probe copies failed"; cat $O/lat_probe_copies.txt; exit 1; }
echo "== QPP_ZERO_COPY=0"; cat $O/lat_probe_copies.txt
timeout -k 10 300 python tools/bench_python_layer.py --packets 16384 > $O/python_layer.json 2> $O/python_layer.err || { echo "python layer failed"; tail -20 $O/python_layer.err; exit 1; }
cat $O/python_layer.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o lat -- python3 tools/lat_trace.py 2000 > $O/lat_trace.log 2>&1 || { echo "trace failed"; tail -20 $O/lat_trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cat {} \;
