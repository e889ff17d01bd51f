#!/bin/bash
# r5i: the library's host path at 1 Mi packets, modes in different orders in
# one process (tools/host_path_probe.py), after the single-device fast path.
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5i; mkdir -p $O
for order in registered staged,registered registered,staged; do
  timeout -k 10 200 python -u tools/host_path_probe.py 1048576 $order > $O/probe_$order.json 2> $O/probe_$order.err || { echo probe failed; tail $O/probe_$order.err; exit 1; }
  echo "$order $(cat $O/probe_$order.json)"
done
