#!/bin/bash
# LDS-array occupancy of a pure-LDS lookup loop (tools/mb_gather.hip, the
# "LDS, 2 VALU per lookup" row) against the GCM kernel: SQ_LDS_IDX_ACTIVE
# per CU-cycle (GRBM_GUI_ACTIVE) is the share of cycles the LDS array works.
#   gpurun -- bash tools/pmc_lds_ceiling.sh
set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_lds
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/mb -o mb -- ./tools/mb_gather > $O/mb.log 2>&1 || { echo mb failed; tail $O/mb.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/ns -o ns -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/ns.log 2>&1 || { echo ns failed; tail $O/ns.log; exit 1; }
for w in mb ns; do
  python3 -c "
import csv,glob,collections
f=glob.glob('$O/$w/*counter_collection.csv')[0]
acc=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name'].split('(')[0]
    if 'k_gcm' in k or 'k_gather' in k: acc[(k,r['Counter_Name'])].append(float(r['Counter_Value']))
ks=sorted({k for k,_ in acc})
for k in ks:
    g=lambda c: sum(acc[(k,c)])/len(acc[(k,c)])
    lds=g('SQ_LDS_IDX_ACTIVE'); gr=g('GRBM_GUI_ACTIVE')
    # GRBM_GUI_ACTIVE sums the 8 XCDs; 32 CUs per XCD
    print('$w', k, 'LDS_IDX_ACTIVE per CU-cycle %.3f' % (lds/(gr/8*256)), 'INSTS_LDS %.4g VALU %.4g' % (g('SQ_INSTS_LDS'), g('SQ_INSTS_VALU')))
"
done
