#!/bin/bash
# r5v: LDS / issue / VALU counters of the final tree, north star (AES-128-GCM)
# and config 3 (ChaCha20-Poly1305), one --pmc pass each
set -uo pipefail
cd $GRAFT_REPO_ROOT
C="SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for cfg in ns 3; do
  bash tools/pmc_one.sh r5v_$cfg "$C" --config $cfg --steps 3 --warmup 2 --cpu-seconds 0 --cpu-all-cores 0 --no-e2e > gpurun_out/pmc_r5v_$cfg.txt 2>&1 || { echo "pmc $cfg failed"; tail -5 gpurun_out/pmc_r5v_$cfg.txt; exit 1; }
  echo "== $cfg"; cat gpurun_out/pmc_r5v_$cfg.txt
done
