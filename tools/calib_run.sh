#!/bin/bash
# Run the HBM counter calibration: timing, then one --pmc pass per counter group.
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/calib; mkdir -p $O
timeout -k 10 60 ./tools/calib_hbm || exit 1
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o f -- ./tools/calib_hbm > $O/f.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o w -- ./tools/calib_hbm > $O/w.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for c in ("f", "w"):
    d = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/calib/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in sorted(d.items()):
        print(k, "per launch KiB", round(sum(v) / len(v)), "-> MB", round(sum(v) / len(v) * 1024 / 1e6, 1))
PY
