#!/bin/bash
# Round 6: host path with the session's D2H by k_d2h (default) against the
# runtime's hipMemcpyAsync D2H (QPP_D2H_KERNEL=0), fresh process each, the
# first process on the box first; then the session / host-path GPU tests.
set -uo pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6m}
O=gpurun_out/$TAG; mkdir -p $O
i=0
for k in 1 0 1 0 1 0; do
  i=$((i+1))
  QPP_D2H_KERNEL=$k timeout -k 10 120 python -u tools/host_trace.py 1048576 4 > $O/host_k${k}_$i.txt 2>&1 || { echo "fail $k"; tail $O/host_k${k}_$i.txt; exit 1; }
  echo "d2h_kernel=$k run $i: $(tail -1 $O/host_k${k}_$i.txt)"
done
grep -h "protect" $O/host_k1_1.txt | head -4
grep -h "protect" $O/host_k0_2.txt | head -4
timeout -k 10 600 python -u -m pytest tests/test_multi_device.py tests/test_gpu_bucketing.py tests/test_batch_io.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
exit $rc
