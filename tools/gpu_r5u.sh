#!/bin/bash
# r5u: host path with the whole process bound to the GPU's NUMA node
# (QPP_PROBE_BIND=1: CPUs, hence first-touch memory and the copy threads)
# against unbound, interleaved, fresh process each, 8 reps per process
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5u; mkdir -p $O
for r in 1 2 3 4; do
  for m in 1 0; do
    QPP_PROBE_BIND=$m QPP_PROBE_REPS=8 timeout -k 10 200 python -u tools/host_path_probe.py 1048576 staged > $O/p_${m}_$r.json 2> $O/p_${m}_$r.err || { echo probe failed; tail $O/p_${m}_$r.err; exit 1; }
    echo "bind=$m $r $(cat $O/p_${m}_$r.json)"
  done
done
