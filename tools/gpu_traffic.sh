#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate runs) over one bench config, then
# tools/traffic.py into gpurun_out/traffic.json.  tools/gpu_traffic.sh TAG CONFIG [PACKETS]
set -uo pipefail
TAG=$1; CFG=$2; PK=${3:-0}
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
ARGS="--config $CFG --packets $PK --steps 3 --warmup 2 --cpu-seconds 0 --cpu-all-cores 0 --no-check --no-e2e ${EXTRA:-}"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- python3 bench.py $ARGS > $O/fetch.log 2>&1 || { echo fetch failed; tail $O/fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- python3 bench.py $ARGS > $O/write.log 2>&1 || { echo write failed; tail $O/write.log; exit 1; }
NAME=$(grep '^{' $O/write.log | tail -1 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['config']['workload'])")
NP=$(grep '^{' $O/write.log | tail -1 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['config']['packets_per_gpu'])")
python3 tools/traffic.py "$NAME" $O/fetch $O/write --packets $NP --out gpurun_out/traffic.json
