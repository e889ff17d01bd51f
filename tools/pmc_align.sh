#!/bin/bash
# WRITE_SIZE / FETCH_SIZE of the GCM kernels with an 11-byte header (ciphertext
# blocks at 11 mod 16) and a 16-byte header (blocks 16-byte aligned).  GPU box.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_align
mkdir -p $O
cd $GRAFT_REPO_ROOT
for h in 11 16; do
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $O/${c}_$h -o pmc -- tools/probe_base 65536 0 bench $h > $O/${c}_$h.log 2>&1
    python3 - $O/${c}_$h $c $h <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_packets" in r["Kernel_Name"] and r["Counter_Name"] == sys.argv[2]:
            d["protect" if "true" in r["Kernel_Name"].split("(")[0] else "unprotect"].append(float(r["Counter_Value"]))
for k, v in sorted(d.items()):
    print(f"hdr {sys.argv[3]} {sys.argv[2]} {k}: {sum(v)/len(v)/1024:.1f} MiB raw per launch ({len(v)} launches)")
PY
  done
done
