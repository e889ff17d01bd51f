#!/bin/bash
# Round 6: host path, D2H by k_xfer, H2D by the copy engines (default) or by
# Round 6: host path, H2D on one stream or alternating over two (QPP_H2D_STREAMS=2), fresh process each.
# Round 6: host path, H2D on one stream or alternating over two (QPP_H2D_STREAMS=2), fresh process each.
set -uo pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6n}
O=gpurun_out/$TAG; mkdir -p $O
i=0
for k in 1 2 1 2 1 2; do
  i=$((i+1))
  QPP_H2D_STREAMS=$k timeout -k 10 120 python -u tools/host_trace.py 1048576 4 > $O/host_h${k}_$i.txt 2>&1 || { echo "fail $k"; tail $O/host_h${k}_$i.txt; exit 1; }
  echo "h2d_streams=$k run $i: $(tail -1 $O/host_h${k}_$i.txt)"
  grep -h "protect" $O/host_h${k}_$i.txt | head -2
done
QPP_H2D_STREAMS=2 timeout -k 10 600 python -u -m pytest tests/test_multi_device.py tests/test_batch_io.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
exit $rc
