#!/bin/bash
# Round 6: the host-buffer path's phase trace at several copy-thread counts
# (NOCOPY=...: the r6i study build's QPP_STUDY_NOCOPY switch, which skipped the
# host copies for timing and has since been removed from the library).
set -uo pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6h}
O=gpurun_out/$TAG; mkdir -p $O
for t in ${THREADS:-6 4 8 12 6}; do
  QPP_COPY_THREADS=$t timeout -k 10 120 python -u tools/host_trace.py 1048576 ${REPS:-5} > $O/host_t$t.txt 2>&1 || { echo "fail $t"; tail $O/host_t$t.txt; exit 1; }
  tail -1 $O/host_t$t.txt
done
for nc in ${NOCOPY:-}; do
  QPP_STUDY_NOCOPY=$nc timeout -k 10 120 python -u tools/host_trace.py 1048576 ${REPS:-5} > $O/host_nc_$nc.txt 2>&1
  echo "nocopy $nc"; grep -v amdgpu.ids $O/host_nc_$nc.txt | head -4
done
cat $O/host_t6.txt
