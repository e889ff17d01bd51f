#!/bin/bash
# r5ar: host copies with non-temporal stores (default) against memcpy
# (QPP_COPY_NT=0): host-buffer parity tests first, then the host-path probe,
# interleaved, fresh process each, 8 call pairs per process
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5ar; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_device.py tests/test_gpu_bucketing.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3 4; do
  for m in 1 0; do
    QPP_COPY_NT=$m QPP_PROBE_REPS=8 timeout -k 10 200 python -u tools/host_path_probe.py 1048576 staged > $O/p_${m}_$r.json 2> $O/p_${m}_$r.err || { echo probe failed; tail $O/p_${m}_$r.err; exit 1; }
    echo "nt=$m $r $(cat $O/p_${m}_$r.json)"
  done
done
