#!/bin/bash
# r5c: GPU tests of the tree (powers region, copy pool), then config 4 (and
# the north star) against variants/powin (the lone kernels' H powers inside
# each slot's tables, 49 KiB stride: round 4's layout), same box, interleaved;
# then the library's host-buffer path (e2e_host_devices) of the tree.
set -uo pipefail
TAG=${1:-r5c}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
for rep in 1 2 3; do
  for v in base powin; do
    if [ "$v" = base ]; then LP=""; else LP="$GRAFT_REPO_ROOT/variants/$v"; fi
    for c in ${CFGS:-4}; do
      LD_LIBRARY_PATH=$LP timeout -k 10 200 python -u bench.py --config $c --steps 20 --warmup 5 --cpu-seconds 0 --cpu-all-cores 0 --no-e2e > $O/b_${c}_${v}_$rep.json 2> $O/b_${c}_${v}_$rep.err || { echo "fail $c $v"; tail -5 $O/b_${c}_${v}_$rep.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/b_${c}_${v}_$rep.json').read().strip().split(chr(10))[-1]); print('$c $v $rep', d['value'], d['kernels_ms'], d['status_ok'])"
    done
  done
done
timeout -k 10 300 python -u -c "
import json, bench
print(json.dumps(bench.e2e_host_devices(bench.CONFIGS['ns'], 0x9001, 1 << 20)))" > $O/e2e_host.json 2> $O/e2e_host.err || { echo e2e failed; tail $O/e2e_host.err; exit 1; }
cat $O/e2e_host.json
timeout -k 10 240 python -u tools/host_dma_probe.py > $O/host_dma_probe.json 2> $O/host_dma_probe.err || { echo dma probe failed; tail $O/host_dma_probe.err; exit 1; }
cat $O/host_dma_probe.json
