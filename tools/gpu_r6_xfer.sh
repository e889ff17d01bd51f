#!/bin/bash
# Round 6: the host path with the copy kernel's workgroup cap (QPP_XFER_WGS)
# and the H2D leg on the copy engines or on k_xfer (QPP_H2D_KERNEL), fresh
# process each, interleaved.
set -uo pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6t}
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  for v in "0 1024" "0 128" "1 32" "1 64" "1 128"; do
    set -- $v
    QPP_H2D_KERNEL=$1 QPP_XFER_WGS=$2 timeout -k 10 120 python -u tools/host_trace.py 1048576 3 > $O/h${1}_w${2}_$rep.txt 2>&1 || { echo "fail $v"; tail $O/h${1}_w${2}_$rep.txt; exit 1; }
    echo "h2d_kernel=$1 wgs=$2 rep $rep: $(tail -1 $O/h${1}_w${2}_$rep.txt)"
    grep -h "protect" $O/h${1}_w${2}_$rep.txt | head -2
  done
done
