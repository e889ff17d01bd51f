#!/bin/bash
# Instruction-fetch counters on the C++ probe harness (GPU box).
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_icache
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY --output-format csv -d $OUT/a -o a -- tools/probe_noprobe > $OUT/a.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d $OUT/b -o b -- tools/probe_noprobe > $OUT/b.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for tag in "ab":
    f = glob.glob(f"/root/repo/gpurun_out/pmc_icache/{tag}/**/*counter_collection.csv", recursive=True)
    if not f: print("no csv", tag); continue
    rows = list(csv.DictReader(open(f[0])))
    agg = collections.defaultdict(float); names = {}
    for r in rows:
        k = (r["Dispatch_Id"], r["Counter_Name"]); agg[k] += float(r["Counter_Value"]); names[r["Dispatch_Id"]] = r["Kernel_Name"][:40]
    for d in sorted({k[0] for k in agg}, key=int):
        print(tag, d, names[d], {c: int(v) for (dd, c), v in agg.items() if dd == d})
PY
