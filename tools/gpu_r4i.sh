#!/bin/bash
# Lone-packet kernels (r4i): GPU tests, then the per-call latency of the object
# API with the lone kernels and with QPP_LONE=0 (quad kernels), the Python
# layer's figures, and a kernel trace of one-packet AEAD.encrypt calls.
#   gpurun -- bash tools/gpu_r4i.sh TAG [skip-tests]
set -uo pipefail
TAG=${1:-r4i}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
if [ "${2:-}" != skip-tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=8 > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
  tail -14 $O/gpu_tests.log
fi
for lone in 1 0; do
  QPP_LONE=$lone timeout -k 10 120 python tools/lat_probe.py > $O/lat_probe_lone$lone.txt 2>&1 || { echo "lat_probe failed"; cat $O/lat_probe_lone$lone.txt; exit 1; }
  echo "== lat_probe QPP_LONE=$lone"; cat $O/lat_probe_lone$lone.txt
done
timeout -k 10 300 python tools/bench_python_layer.py --packets 16384 > $O/python_layer.json 2> $O/python_layer.err || { echo "python layer failed"; tail -20 $O/python_layer.err; exit 1; }
cat $O/python_layer.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o lat -- python3 tools/lat_trace.py 2000 > $O/lat_trace.log 2>&1 || { echo "trace failed"; tail -20 $O/lat_trace.log; exit 1; }
cat $O/lat_trace.log | tail -3
find $O/trace -name "*kernel_stats.csv" -exec cat {} \;
