#!/bin/bash
# ChaCha20-Poly1305 fixed-work study (r4h): GPU tests, then same-box A/B of
# the tree against variants/$2 (config 3 at 64 Ki and 1 Mi, interleaved),
# then the payload-size sweep (time, SQ_INSTS_VALU) for both libraries.
#   gpurun -- bash tools/gpu_r4h.sh TAG VARIANT [skip-tests]
set -uo pipefail
TAG=${1:-r4h}; V=${2:-r4head}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
if [ "${3:-}" != skip-tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
fi
for p in 0 1048576; do
  CFG=3 PKTS=$p bash tools/ab_lib.sh $V > $O/ab_c3_$p.txt 2>&1 || { echo "ab $p failed"; cat $O/ab_c3_$p.txt; exit 1; }
  echo "== config 3 packets $p"; cat $O/ab_c3_$p.txt
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for lib in base $V; do
  if [ $lib = base ]; then LP=$GRAFT_REPO_ROOT/aioquic_amd; else LP=$GRAFT_REPO_ROOT/variants/$V; fi
  LD_LIBRARY_PATH=$LP timeout -k 5 120 tools/chacha_sizes 2 65536 > $O/sizes_$lib.log 2>&1 || { echo "sizes $lib failed"; cat $O/sizes_$lib.log; exit 1; }
  echo "== sizes $lib"; cat $O/sizes_$lib.log
  LD_LIBRARY_PATH=$LP timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/pmc_$lib -o p -- tools/chacha_sizes 2 65536 > $O/pmc_$lib.log 2>&1 || { echo "pmc $lib failed"; tail -5 $O/pmc_$lib.log; exit 1; }
done
python3 - $O $V <<'PY'
import csv, glob, sys, collections
for lib in ("base", sys.argv[2]):
    rows = collections.defaultdict(dict); names = {}
    for f in glob.glob(f"{sys.argv[1]}/pmc_{lib}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_chacha" in r["Kernel_Name"]:
                d = int(r["Dispatch_Id"]); rows[d][r["Counter_Name"]] = float(r["Counter_Value"])
                names[d] = "protect" if "true" in r["Kernel_Name"].split("(")[0] else "unprotect"
    ids = sorted(rows); per = 46
    for s, size in enumerate([53, 245, 501, 757, 1173]):
        blk = ids[s * per:(s + 1) * per]
        for kind in ("protect", "unprotect"):
            ks = [d for d in blk if names[d] == kind][3:]
            if ks:
                d = ks[len(ks) // 2]
                print(lib, size, kind, " ".join(f"{c}={v:.6g}" for c, v in sorted(rows[d].items())))
PY
