#!/bin/bash
# r4y: GPU tests, then object-API latency of the lone kernels reading a
# staged call from LDS (this tree) against the previous engine (variants/head,
# staged call copied to device memory), same box, interleaved; launch floor.
set -uo pipefail
TAG=${1:-r4y}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for rep in 1 2 3; do
  for v in lds head; do
    lp=""; [[ $v == head ]] && lp=$PWD/variants/head
    LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 120 python tools/lat_probe.py > $O/lat_${v}_$rep.txt 2>&1 || { echo "lat_probe failed ($v)"; cat $O/lat_${v}_$rep.txt; exit 1; }
    echo "== $v rep $rep"; grep us $O/lat_${v}_$rep.txt
  done
done
for v in lds head; do
  lp=""; [[ $v == head ]] && lp=$PWD/variants/head
  LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 300 python tools/bench_python_layer.py --packets 16384 > $O/python_layer_$v.json 2> $O/python_layer_$v.err || { echo "python layer failed"; tail -20 $O/python_layer_$v.err; exit 1; }
  echo "== python layer $v"; python -c "import json; d=json.load(open('$O/python_layer_$v.json')); print(json.dumps(d.get('latency_us', d)))"
done
timeout -k 10 60 tools/launch_floor > $O/launch_floor.txt 2>&1 && cat $O/launch_floor.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o lat -- python3 tools/lat_trace.py 2000 > $O/lat_trace.log 2>&1 || { echo "trace failed"; tail -20 $O/lat_trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cat {} \;
# the table fill (load_te) changed for the quad kernels too: config 2 and the
# north star against the previous engine, interleaved
NOTEST=1 bash tools/gpu_ab2.sh r4y_ab 2 ns 2 ns 3 -- head
