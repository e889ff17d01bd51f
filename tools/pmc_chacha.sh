#!/bin/bash
# Where the ChaCha20-Poly1305 kernel's wave cycles go (1 Mi and 64 Ki protect):
# one --pmc pass of 8 SQ counters + GRBM_GUI_ACTIVE per size.
#   gpurun -- bash tools/pmc_chacha.sh TAG
set -uo pipefail
TAG=${1:-ch}
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
for n in 1048576 65536; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/n$n -o p -- python3 bench.py --config 3 --packets $n --steps 3 --warmup 1 --cpu-seconds 0 --no-check > $O/n$n.log 2>&1 || { echo "n=$n failed"; tail -5 $O/n$n.log; exit 1; }
  python3 - $O/n$n $n <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_chacha" in r["Kernel_Name"]:
            d[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(d.items()):
    print(sys.argv[2], k, c, "%.4g" % (sum(v) / len(v)))
PY
done
