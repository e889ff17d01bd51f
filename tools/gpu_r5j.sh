#!/bin/bash
# r5j: registered host path by hipHostRegister flags (QPP_REG_FLAGS), fresh process each
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5j; mkdir -p $O
for f in 0x1 0x0 0x8 0x9 0x2; do
  QPP_REG_FLAGS=$f timeout -k 10 200 python -u tools/host_path_probe.py 1048576 registered > $O/probe_$f.json 2> $O/probe_$f.err || { echo probe failed; tail $O/probe_$f.err; exit 1; }
  echo "$f $(cat $O/probe_$f.json)"
done
timeout -k 10 200 python -u tools/host_path_probe.py 1048576 staged > $O/probe_staged.json 2> $O/probe_staged.err && echo "staged $(cat $O/probe_staged.json)"
