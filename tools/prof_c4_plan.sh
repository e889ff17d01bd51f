#!/bin/bash
# Round 6: rocprofv3 kernel trace of config 4 (bucketed AES-256-GCM, 4096 keys): the plan kernels' share of a step.
#   gpurun -- bash tools/prof_c4_plan.sh TAG
set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e --sustain-seconds 0 > $O/kt.log 2>&1 || { echo "rocprof failed"; tail $O/kt.log; exit 1; }
f=$(ls $O/kt/*kernel_stats.csv | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in rows: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['TotalDurationNs'], r['Percentage'])
" | tee $O/stats.txt
