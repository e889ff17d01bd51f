#!/bin/bash
# r5p: box topology; the pipelined session tests (tapered chunks); the
# library's host path with the taper (probe, three runs)
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5p; mkdir -p $O
{ lscpu | head -24; for f in /sys/class/drm/card*/device/numa_node; do echo "$f $(cat $f)"; done; ls /sys/devices/system/node/; cat /sys/devices/system/node/node*/cpulist; python3 -c "import os; a=sorted(os.sched_getaffinity(0)); print('affinity', len(a), a)"; } > $O/topology.txt 2>&1
grep -E "Socket|NUMA|Model name|affinity|node" $O/topology.txt | head -20
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_device.py -k "session or multi" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  QPP_SESSION_TRACE=1 timeout -k 10 200 python -u tools/host_path_probe.py 1048576 staged > $O/probe$r.json 2> $O/probe$r.err || { echo probe failed; tail $O/probe$r.err; exit 1; }
  echo "$(cat $O/probe$r.json) $(grep 'qpp session' $O/probe$r.err | tail -1)"
done
