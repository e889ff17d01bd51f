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
# size sweep through the C ABI (64 Ki packets, payloads 53..1173 B): time and
# counters per launch, protect and unprotect alternating, 23 launches per size
LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/aioquic_amd timeout -k 5 120 tools/chacha_sizes 2 65536 > $O/sizes.log 2>&1 || { echo "sizes failed"; cat $O/sizes.log; exit 1; }
cat $O/sizes.log
LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/aioquic_amd timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/sz -o p -- tools/chacha_sizes 2 65536 > $O/sz.log 2>&1 || { echo "sizes pmc failed"; tail -5 $O/sz.log; exit 1; }
python3 - $O/sz <<'PY'
import csv, glob, sys, collections
rows = collections.defaultdict(dict)
names = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_chacha" in r["Kernel_Name"]:
            d = int(r["Dispatch_Id"])
            rows[d][r["Counter_Name"]] = float(r["Counter_Value"])
            names[d] = "protect" if "true" in r["Kernel_Name"].split("(")[0] else "unprotect"
ids = sorted(rows)
# 5 sizes x 23 iterations x 2 launches, in order; report the median launch of each size/direction
per = 46
sizes = [53, 245, 501, 757, 1173]
for s, size in enumerate(sizes):
    blk = ids[s * per:(s + 1) * per]
    for kind in ("protect", "unprotect"):
        ks = [d for d in blk if names[d] == kind][3:]
        if not ks: continue
        d = ks[len(ks) // 2]
        print(size, kind, " ".join(f"{c}={v:.4g}" for c, v in sorted(rows[d].items())))
PY
