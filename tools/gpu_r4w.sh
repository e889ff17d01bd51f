#!/bin/bash
# r4w: GPU tests, then object-API latency with the small-call completion
# polled (default) and with the runtime's blocking wait (QPP_SPIN_WAIT=0),
# same box, interleaved; the Python layer's per-call figures for both.
set -uo pipefail
TAG=${1:-r4w}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for rep in 1 2; do
  for sw in 1 0; do
    QPP_SPIN_WAIT=$sw timeout -k 10 120 python tools/lat_probe.py > $O/lat_spin${sw}_$rep.txt 2>&1 || { echo "lat_probe failed"; cat $O/lat_spin${sw}_$rep.txt; exit 1; }
    echo "== QPP_SPIN_WAIT=$sw rep $rep"; grep us $O/lat_spin${sw}_$rep.txt
  done
done
for sw in 1 0; do
  QPP_SPIN_WAIT=$sw timeout -k 10 300 python tools/bench_python_layer.py --packets 16384 > $O/python_layer_spin$sw.json 2> $O/python_layer_spin$sw.err || { echo "python layer failed"; tail -20 $O/python_layer_spin$sw.err; exit 1; }
  echo "== python layer QPP_SPIN_WAIT=$sw"; python -c "import json,sys; d=json.load(open('$O/python_layer_spin$sw.json')); print(json.dumps(d.get('latency_us', d)))"
done
