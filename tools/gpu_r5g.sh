#!/bin/bash
# r5g: D2H engine probe; the library's host path with D2H by the copy engines
# (default) and by the runtime's blit kernels (QPP_D2H=blit); the GPU tests
# touching the host path; then the synthesized-descriptor bound (variants/synth).
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5g; mkdir -p $O
timeout -k 10 200 python -u tools/d2h_engine_probe.py > $O/d2h_engine_probe.json 2>&1 || { echo d2h probe failed; tail $O/d2h_engine_probe.json; exit 1; }
tail -1 $O/d2h_engine_probe.json
timeout -k 10 300 python -u -m pytest tests/test_multi_device.py tests/test_gpu_parity.py -k "session or multi or registered" -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in engines blit; do
  if [ $m = blit ]; then E="QPP_D2H=blit"; else E="QPP_D2H=engines"; fi
  env $E timeout -k 10 200 python -u tools/host_path_probe.py > $O/host_$m.json 2> $O/host_$m.err || { echo host probe failed; tail $O/host_$m.err; exit 1; }
  echo "$m $(cat $O/host_$m.json)"
done
bash tools/gpu_ab5.sh r5g_ab ns synth
