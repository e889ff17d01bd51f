#!/bin/bash
# r5e: where the library's host-buffer path spends its time: the probe plain,
# then under rocprofv3 (kernel trace + memory-copy trace, no counters).
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5e; mkdir -p $O
timeout -k 10 200 python -u tools/host_path_probe.py > $O/probe.json 2> $O/probe.err || { echo probe failed; tail $O/probe.err; exit 1; }
cat $O/probe.json
cd /tmp && export TMPDIR=/tmp
for m in staged registered; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/tr_$m -o tr -- python3 $GRAFT_REPO_ROOT/tools/host_path_probe.py 262144 $m > $O/tr_$m.log 2>&1 || { echo "trace $m failed"; tail $O/tr_$m.log; exit 1; }
  tail -1 $O/tr_$m.log
  find $O/tr_$m -name '*stats*.csv' | head
done
