#!/bin/bash
# r4zb: GPU tests; the one-packet kernel's phases (tools/lone_probe); object-API
# latency of this tree against the previous engine (variants/head), same box,
# interleaved; k_lone_gcm durations under rocprofv3.
set -uo pipefail
TAG=${1:-r4zb}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
[ -n "${NOTEST:-}" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 tools/lone_probe 400 ${PROBE_SUITE:-0} > $O/lone_probe.txt 2>&1 || { echo "lone_probe failed"; cat $O/lone_probe.txt; exit 1; }
cat $O/lone_probe.txt
lp_of() { [[ $1 == new ]] && echo "" || echo "$PWD/variants/$1"; }
for rep in 1 2 3; do
  for v in new head; do
    LD_LIBRARY_PATH=$(lp_of $v) timeout -k 10 120 python tools/lat_probe.py > $O/lat_${v}_$rep.txt 2>&1 || { echo "lat_probe failed ($v)"; cat $O/lat_${v}_$rep.txt; exit 1; }
    echo "== $v rep $rep: $(grep us $O/lat_${v}_$rep.txt | tr '\n' ' ')"
  done
done
for v in new head; do
  LD_LIBRARY_PATH=$(lp_of $v) timeout -k 10 300 python tools/bench_python_layer.py --packets 16384 > $O/python_layer_$v.json 2> $O/python_layer_$v.err || { echo "python layer failed"; tail -20 $O/python_layer_$v.err; exit 1; }
  echo "== python layer $v"; python -c "import json; d=json.load(open('$O/python_layer_$v.json')); print(json.dumps(d.get('latency_us', d)))"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in new head; do
  LD_LIBRARY_PATH=$(lp_of $v) timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o lat -- python3 tools/lat_trace.py 2000 > $O/lat_trace_$v.log 2>&1 || { echo "trace failed"; tail -20 $O/lat_trace_$v.log; exit 1; }
  echo "== $v: $(find $O/trace_$v -name '*kernel_stats.csv' -exec grep k_lone {} \; | awk -F'",' '{print $2}' | cut -d, -f1-6)"
done
# the table fill (load_te) is shared with the quad kernels: config 2 and the
# north star against the previous engine, interleaved
[ -n "${NOBENCH:-}" ] || NOTEST=1 bash tools/gpu_ab2.sh ${TAG}_ab 2 ns 2 ns -- head
