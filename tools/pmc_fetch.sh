#!/bin/bash
# FETCH_SIZE of tools/mb_fetch's grouped and random read orders (1 Mi x 1189 B
# read), one PMC pass per counter set.   gpurun -- bash tools/pmc_fetch.sh
set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 5 60 tools/mb_fetch || exit 1
i=0
for C in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $O/p$i -o p$i -- tools/mb_fetch > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  python3 - $O/p$i <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(d.items()):
    x = sum(v) / len(v)
    extra = f"  = {x*1024/1e9:.3f} GB raw, {x*1024/1.2468e9:.3f}x the bytes read" if c == "FETCH_SIZE" else ""
    print(f"{k:24s} {c:24s} {x:.4g}{extra}")
PY
done
