#!/bin/bash
# Counter A/B on one bench config: kernel trace + the LDS / wait counter pass
# for the in-tree library and each variants/<name>/ build.
#   tools/gpu_prof_ab.sh TAG CONFIG [variant...]
set -uo pipefail
TAG=$1; CFG=$2; shift 2
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
ARGS="--config $CFG --packets ${PKTS:-0} --steps 3 --warmup 2 --cpu-seconds 0 --cpu-all-cores 0"
for v in base "$@"; do
  O=$GRAFT_REPO_ROOT/gpurun_out/$TAG/$v
  mkdir -p $O
  if [ "$v" = base ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH="$GRAFT_REPO_ROOT/variants/$v"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py $ARGS > $O/kt.log 2>&1 || { echo "kt failed $v"; tail $O/kt.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc1 -o pmc1 -- python3 bench.py $ARGS > $O/pmc1.log 2>&1 || { echo "pmc1 failed $v"; tail $O/pmc1.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VALU --output-format csv -d $O/pmc2 -o pmc2 -- python3 bench.py $ARGS > $O/pmc2.log 2>&1 || { echo "pmc2 failed $v"; tail $O/pmc2.log; exit 1; }
  python3 tools/prof_summary.py $O > $O/summary.md && echo "== $v" && grep -E "k_gcm|k_packets|k_chacha" $O/summary.md
done
