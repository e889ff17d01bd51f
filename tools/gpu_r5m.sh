#!/bin/bash
# r5m: registered host path by D2H mode (QPP_REG_D2H 0/1/2), staged path by copy threads
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5m; mkdir -p $O
for m in 1 0 2; do
  QPP_REG_D2H=$m QPP_SESSION_TRACE=1 timeout -k 10 200 python -u tools/host_path_probe.py 1048576 registered > $O/probe_d$m.json 2> $O/probe_d$m.err || { echo probe failed; tail $O/probe_d$m.err; exit 1; }
  echo "reg_d2h $m $(cat $O/probe_d$m.json) $(grep 'qpp session' $O/probe_d$m.err | tail -1)"
done
for t in 4 2 6 8; do
  QPP_COPY_THREADS=$t timeout -k 10 200 python -u tools/host_path_probe.py 1048576 staged > $O/probe_t$t.json 2> $O/probe_t$t.err || { echo probe failed; tail $O/probe_t$t.err; exit 1; }
  echo "threads $t $(cat $O/probe_t$t.json)"
done
