#!/bin/bash
# r4z: object-API latency, three engines on one box, interleaved: this tree
# (staged call read from LDS), variants/dev (table fill unrolled, staged call
# through device memory), variants/head (previous engine); then each one's
# k_lone_gcm duration under rocprofv3.
set -uo pipefail
TAG=${1:-r4z}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
lp_of() { [[ $1 == lds ]] && echo "" || echo "$PWD/variants/$1"; }
for rep in 1 2 3; do
  for v in lds dev head; do
    LD_LIBRARY_PATH=$(lp_of $v) timeout -k 10 120 python tools/lat_probe.py > $O/lat_${v}_$rep.txt 2>&1 || { echo "lat_probe failed ($v)"; cat $O/lat_${v}_$rep.txt; exit 1; }
    echo "== $v rep $rep: $(grep us $O/lat_${v}_$rep.txt | tr '\n' ' ')"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in lds dev head; do
  LD_LIBRARY_PATH=$(lp_of $v) timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o lat -- python3 tools/lat_trace.py 2000 > $O/lat_trace_$v.log 2>&1 || { echo "trace failed"; tail -20 $O/lat_trace_$v.log; exit 1; }
  echo "== $v: $(find $O/trace_$v -name '*kernel_stats.csv' -exec grep k_lone {} \; | cut -d, -f1,4,6,7 | cut -c1-40,200-)"
done
