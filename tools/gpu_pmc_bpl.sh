#!/bin/bash
# PMC passes (one counter group per run) on the north-star bench for GCM
# blocks-per-lane 1 and 2.
set -uo pipefail
cd $GRAFT_REPO_ROOT
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE"
B="SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
for b in ${BPLS:-1 2}; do
  for g in A B FETCH_SIZE WRITE_SIZE; do
    case $g in A) C=$A;; B) C=$B;; *) C=$g;; esac
    QPP_GCM_BPL=$b bash tools/pmc_one.sh bpl${b}_$g "$C" --steps 3 --warmup 2 --cpu-seconds 0 --cpu-all-cores 0 > gpurun_out/pmc_bpl${b}_$g.txt 2>&1 || { echo "pmc $b $g failed"; cat gpurun_out/pmc_bpl${b}_$g.txt | tail -5; exit 1; }
    echo "== bpl $b $g"; cat gpurun_out/pmc_bpl${b}_$g.txt
  done
done
