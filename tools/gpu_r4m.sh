#!/bin/bash
# r4m: GPU tests, the object-API latency (lone kernels, output written into
# the pinned staging), and a same-box A/B of the GCM start-up change (the
# first slot's GHASH entry loaded beside the AES image) against
# variants/$2 at configs 2, ns, 4 (interleaved, tools/ab_lib.sh).
#   gpurun -- bash tools/gpu_r4m.sh TAG VARIANT
set -uo pipefail
TAG=${1:-r4m}; V=${2:-prec2}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python tools/lat_probe.py > $O/lat_probe.txt 2>&1 || { echo "lat_probe failed"; cat $O/lat_probe.txt; exit 1; }
cat $O/lat_probe.txt
timeout -k 10 300 python tools/bench_python_layer.py --packets 16384 > $O/python_layer.json 2> $O/python_layer.err || { echo "python layer failed"; tail -20 $O/python_layer.err; exit 1; }
cat $O/python_layer.json
for c in 2 ns 2 4; do
  CFG=$c bash tools/ab_lib.sh $V > $O/ab_c$c.txt 2>&1 || { echo "ab $c failed"; cat $O/ab_c$c.txt; exit 1; }
  echo "== config $c"; cat $O/ab_c$c.txt
done
