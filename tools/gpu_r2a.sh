#!/bin/bash
# Round-2 probe pass: building-block microbenchmarks with the measured clock,
# then LDS / wait counters and the clock on the 1 Mi protect kernel.
set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2a
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 150 ./tools/mb_aes > $O/mb_aes.log 2>&1 || { echo "mb_aes failed"; cat $O/mb_aes.log; exit 1; }
cat $O/mb_aes.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ARGS="--packets 1048576 --steps 3 --warmup 2 --cpu-seconds 0"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py $ARGS > $O/kt.log 2>&1 || { echo kt failed; tail $O/kt.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc1 -o pmc1 -- python3 bench.py $ARGS > $O/pmc1.log 2>&1 || { echo pmc1 failed; tail $O/pmc1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VALU --output-format csv -d $O/pmc2 -o pmc2 -- python3 bench.py $ARGS > $O/pmc2.log 2>&1 || { echo pmc2 failed; tail $O/pmc2.log; exit 1; }
python3 tools/prof_summary.py $O > $O/summary.md && cat $O/summary.md
