#!/bin/bash
# rocprofv3 passes over a short bench run (GPU box).  Usage: tools/profile.sh TAG [bench args]
# Pass 1: kernel trace + stats.  Passes 2-4: PMC counters, one group per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -euo pipefail
TAG=${1:-r1}; shift || true
ARGS=${*:-"--steps 5 --warmup 2 --cpu-seconds 0"}
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py $ARGS > $OUT/kt.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc1 -o pmc1 -- python3 bench.py $ARGS > $OUT/pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc2 -o pmc2 -- python3 bench.py $ARGS > $OUT/pmc2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc3 -o pmc3 -- python3 bench.py $ARGS > $OUT/pmc3.log 2>&1
echo profile-done $TAG
