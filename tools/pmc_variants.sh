#!/bin/bash
# WRITE_SIZE per GCM launch for probe variants (GPU box): tools/pmc_variants.sh v1 v2 ...
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_var
mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$v -o pmc -- tools/probe_$v 65536 0 bench > $O/$v.log 2>&1
  python3 - $O/$v $v <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_packets" in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE":
            d["protect" if "true" in r["Kernel_Name"].split("(")[0] else "unprotect"].append(float(r["Counter_Value"]))
print(sys.argv[2], " ".join(f"{k} WRITE_SIZE {sum(v)/len(v)/1024:.1f} MiB" for k, v in sorted(d.items())))
PY
done
