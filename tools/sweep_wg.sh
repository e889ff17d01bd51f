#!/bin/bash
# Workgroup-size sweep of the packet kernels (GPU box).  Prints one JSON line per variant.
set -uo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in ${CONFIGS:-2 3}; do
  for wg in 512 768 1024; do
    if [ "$cfg" = "3" ]; then export QPP_WG_CHACHA=$wg; unset QPP_WG_GCM; else export QPP_WG_GCM=$wg; unset QPP_WG_CHACHA; fi
    timeout -k 10 120 python bench.py --config $cfg --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/sweep_${cfg}_${wg}.json 2>/dev/null || { echo "fail cfg=$cfg wg=$wg"; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/sweep_${cfg}_${wg}.json')); print('cfg', $cfg, 'wg', $wg, d['value'], d['kernels_ms'], d['status_ok'])"
  done
done
