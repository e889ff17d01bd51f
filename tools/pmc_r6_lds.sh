#!/bin/bash
# Round 6: the LDS pipeline's back-pressure counters of the GCM kernel at the
# north star (tools/pv_base, bench mode), one --pmc pass.
set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/pmc -o pmc -- $GRAFT_REPO_ROOT/tools/pv_base 1048576 0 bench > $O/pmc.log 2>&1 || { echo pmc failed; tail $O/pmc.log; exit 1; }
C2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_IFETCH GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C2 --output-format csv -d $O/pmc2 -o pmc -- $GRAFT_REPO_ROOT/tools/pv_base 1048576 0 bench > $O/pmc2.log 2>&1 || { echo pmc2 failed; tail $O/pmc2.log; exit 1; }
cd $GRAFT_REPO_ROOT
for d in pmc pmc2; do
python3 -c "
import csv,glob,collections
f=glob.glob('$O/$d/**/*counter_collection.csv', recursive=True)[0]
acc=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name'].split('(')[0]
    if 'k_gcm' in k: acc[(k,r['Counter_Name'])].append(float(r['Counter_Value']))
for (k,c) in sorted(acc):
    v=sorted(acc[(k,c)]); print(k, c, len(v), '%.5g' % v[len(v)//2])
"
done
