#!/bin/bash
# r5q: host path, copy threads on the GPU's NUMA node (default) vs anywhere
# (QPP_COPY_NUMA=0), interleaved, fresh process each
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5q; mkdir -p $O
for r in 1 2 3; do
  for m in 1 0; do
    QPP_COPY_NUMA=$m QPP_SESSION_TRACE=1 timeout -k 10 200 python -u tools/host_path_probe.py 1048576 staged > $O/p_${m}_$r.json 2> $O/p_${m}_$r.err || { echo probe failed; tail $O/p_${m}_$r.err; exit 1; }
    echo "numa=$m $r $(cat $O/p_${m}_$r.json) $(grep 'qpp session' $O/p_${m}_$r.err | tail -1)"
  done
done
