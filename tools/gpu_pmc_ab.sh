#!/bin/bash
# One LDS/issue counter pass on the north-star bench for the in-tree library
# and for variants/<name> builds: tools/gpu_pmc_ab.sh variant...
set -uo pipefail
cd $GRAFT_REPO_ROOT
C="SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for v in base "$@"; do
  if [ "$v" = base ]; then LP=""; else LP="$GRAFT_REPO_ROOT/variants/$v"; fi
  LD_LIBRARY_PATH=$LP bash tools/pmc_one.sh ab_$v "$C" --config ${CFG:-ns} --steps 3 --warmup 2 --cpu-seconds 0 --cpu-all-cores 0 > gpurun_out/pmc_ab_$v.txt 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/pmc_ab_$v.txt; exit 1; }
  echo "== $v"; grep "true" gpurun_out/pmc_ab_$v.txt
done
