#!/bin/bash
# r5l: host phases of the pipelined session (QPP_SESSION_TRACE=1), 1 Mi
# packets, staged then registered; copy threads 8 vs 16 on the staged path
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5l; mkdir -p $O
QPP_SESSION_TRACE=1 timeout -k 10 200 python -u tools/host_path_probe.py 1048576 staged,registered > $O/probe.json 2> $O/probe.err || { echo probe failed; tail $O/probe.err; exit 1; }
cat $O/probe.json; grep "qpp session" $O/probe.err | tail -12
for t in 8 16 4; do
  QPP_COPY_THREADS=$t timeout -k 10 200 python -u tools/host_path_probe.py 1048576 staged > $O/probe_t$t.json 2> $O/probe_t$t.err || { echo probe failed; tail $O/probe_t$t.err; exit 1; }
  echo "threads $t $(cat $O/probe_t$t.json)"
done
