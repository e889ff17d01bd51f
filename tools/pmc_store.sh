#!/bin/bash
# WRITE_SIZE of tools/mb_store's three output patterns (one PMC pass each
# counter set).   gpurun -- bash tools/pmc_store.sh
set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_store
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 5 60 tools/mb_store || exit 1
i=0
for C in "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $O/p$i -o p$i -- tools/mb_store > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  python3 - $O/p$i <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(d.items()):
    print(f"{k:28s} {c:24s} {sum(v)/len(v):.4g} per launch ({len(v)} launches)")
PY
done
