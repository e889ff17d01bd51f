#!/bin/bash
# Workgroup-size sweep of the packet kernels (GPU box).  One line per variant.
#   CFG=3 tools/sweep_wg.sh   (ChaCha: QPP_WG_CHACHA_ENC/DEC in 256 512 1024)
#   CFG=2 tools/sweep_wg.sh   (GCM: QPP_WG_GCM in 512 768 1024)
set -uo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=${CFG:-3}
if [ "$CFG" = 3 ]; then SIZES="256 512 1024"; VARS="QPP_WG_CHACHA_ENC QPP_WG_CHACHA_DEC"; else SIZES="512 768 1024"; VARS="QPP_WG_GCM"; fi
for wg in $SIZES; do
  for v in $VARS; do export $v=$wg; done
  timeout -k 10 120 python bench.py --config $CFG --steps 30 --warmup 3 --cpu-seconds 0 > gpurun_out/sweep_${CFG}_${wg}.json 2>/dev/null || { echo "fail cfg=$CFG wg=$wg"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sweep_${CFG}_${wg}.json')); print('cfg', $CFG, 'wg', $wg, d['value'], d['kernels_ms'], d['status_ok'])"
done
