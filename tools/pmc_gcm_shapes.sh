#!/bin/bash
# SQ counters of the GCM kernel at the north star under both workgroup shapes
# (one 1024-thread workgroup per CU, and QPP_GCM_WG2=1: two of 512).
#   gpurun -- bash tools/pmc_gcm_shapes.sh TAG
set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/wg1 -o wg1 -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --cpu-all-cores 0 --no-check > $O/wg1.log 2>&1 || { echo wg1 failed; tail $O/wg1.log; exit 1; }
QPP_GCM_WG2=1 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/wg2 -o wg2 -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --cpu-all-cores 0 --no-check > $O/wg2.log 2>&1 || { echo wg2 failed; tail $O/wg2.log; exit 1; }
for w in wg1 wg2; do
  python3 -c "
import csv,glob,collections
f=glob.glob('$O/$w/*counter_collection.csv')[0]
acc=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name'].split('(')[0]
    if 'k_gcm' in k: acc[(k,r['Counter_Name'])].append(float(r['Counter_Value']))
for k in sorted({k for k,_ in acc}):
    g=lambda c: sorted(acc[(k,c)])[len(acc[(k,c)])//2]
    gr=g('GRBM_GUI_ACTIVE')/8; cu=gr*256
    print('$w', k, 'cycles/XCD %.3g' % gr, 'LDS_IDX_ACTIVE/CU-cycle %.3f' % (g('SQ_LDS_IDX_ACTIVE')/cu),
          'INSTS_LDS %.4g VALU %.4g' % (g('SQ_INSTS_LDS'), g('SQ_INSTS_VALU')),
          'WAIT_INST_LDS/WAVE_CYCLES %.3f WAIT_ANY/WAVE_CYCLES %.3f' % (g('SQ_WAIT_INST_LDS')/g('SQ_WAVE_CYCLES'), g('SQ_WAIT_ANY')/g('SQ_WAVE_CYCLES')),
          'BUSY %.3g' % g('SQ_BUSY_CYCLES'))
"
done
