#!/bin/bash
# r4x: object-API latency under HIP runtime settings (kernel arguments in
# device memory, a longer active wait before the interrupt), same box,
# interleaved; nothing in the library changes.
set -uo pipefail
TAG=${1:-r4x}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  for cfg in base HIP_FORCE_DEV_KERNARG=1 ROC_ACTIVE_WAIT_TIMEOUT=100 HIP_FORCE_DEV_KERNARG=1,ROC_ACTIVE_WAIT_TIMEOUT=100; do
    envs=""; [[ $cfg != base ]] && envs=${cfg//,/ }
    f=$O/lat_${cfg//[=,]/_}_$rep.txt
    env $envs timeout -k 10 120 python tools/lat_probe.py > $f 2>&1 || { echo "lat_probe failed ($cfg)"; cat $f; exit 1; }
    echo "== $cfg rep $rep"; grep us $f
  done
done
