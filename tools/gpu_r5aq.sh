#!/bin/bash
# r5aq: host path with every page of the process interleaved over the NUMA
# nodes (QPP_PROBE_INTERLEAVE=1) against the default first-touch placement,
# interleaved, fresh process each, 8 call pairs per process
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5aq; mkdir -p $O
for r in 1 2 3 4; do
  for m in 1 0; do
    QPP_PROBE_INTERLEAVE=$m QPP_PROBE_REPS=8 timeout -k 10 200 python -u tools/host_path_probe.py 1048576 staged > $O/p_${m}_$r.json 2> $O/p_${m}_$r.err || { echo probe failed; tail $O/p_${m}_$r.err; exit 1; }
    echo "interleave=$m $r $(cat $O/p_${m}_$r.json) $(grep -h 'interleave over' $O/p_${m}_$r.err)"
  done
done
