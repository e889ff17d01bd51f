#!/bin/bash
# r5h: the library's host path at 256 Ki and 1 Mi packets, staged and
# registered, then a rocprofv3 timeline (kernel + memory-copy trace) of the
# 1 Mi registered run.
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5h; mkdir -p $O
for n in 262144 1048576; do
  timeout -k 10 200 python -u tools/host_path_probe.py $n > $O/probe_$n.json 2> $O/probe_$n.err || { echo probe failed; tail $O/probe_$n.err; exit 1; }
  echo "$n $(cat $O/probe_$n.json)"
done
cd /tmp && export TMPDIR=/tmp
for m in registered staged; do
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr_$m -o tr -- python3 $GRAFT_REPO_ROOT/tools/host_path_probe.py 1048576 $m > $O/tr_$m.log 2>&1 || { echo "trace failed"; tail $O/tr_$m.log; exit 1; }
grep gib_s $O/tr_$m.log | tail -1
done
