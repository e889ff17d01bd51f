#!/bin/bash
# One --pmc pass over a short bench run (GPU box).  Usage: tools/pmc_one.sh TAG "COUNTERS" [bench args]
set -euo pipefail
TAG=$1; CNT=$2; shift 2
ARGS=${*:-"--steps 5 --warmup 2 --cpu-seconds 0"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc $CNT --output-format csv -d $OUT -o pmc -- python3 bench.py $ARGS > $OUT/log 2>&1
python3 - $OUT <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in ("k_gcm", "k_chacha", "k_packets")):
            d[(r["Kernel_Name"].split("(")[0][-30:], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(d.items()):
    print(k, len(v), sum(v) / len(v))
PY
