#!/bin/bash
# Instruction mix of the packet kernels (one PMC pass per workload; counters
# fit one SQ block of 8).   gpurun -- bash tools/pmc_mix.sh TAG
set -uo pipefail
TAG=${1:-mix}
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/c3 -o c3 -- python3 bench.py --config 3 --packets 1048576 --steps 3 --warmup 1 --cpu-seconds 0 > $O/c3.log 2>&1 || { echo c3 failed; tail $O/c3.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/ns -o ns -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/ns.log 2>&1 || { echo ns failed; tail $O/ns.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/pmc_" + os.environ.get("TAG", "mix")
PY
for w in c3 ns; do
  python3 -c "
import csv,glob,collections,sys
f=glob.glob('$O/$w/*counter_collection.csv')[0]
acc=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name'].split('(')[0]
    if 'k_gcm' in k or 'k_chacha' in k: acc[(k,r['Counter_Name'])].append(float(r['Counter_Value']))
for (k,c),v in sorted(acc.items()): print('$w', k, c, '%.4g' % (sum(v)/len(v)))
"
done
