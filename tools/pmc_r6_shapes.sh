#!/bin/bash
# Round 6: the two GCM launch shapes at the north star, one 1024-thread
# workgroup per CU (tools/pv_base) against two of 512 with the launch-wide item
# pool (tools/pv_w512p): SQ counters in one --pmc pass each, and the phase
# probe of both (tools/probe, tools/probe_w512).
#   gpurun -- bash tools/pmc_r6_shapes.sh TAG
set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in base w512p; do
  timeout -k 5 60 ./tools/pv_$v 1048576 0 bench > $O/bench_$v.txt 2>&1 || exit 1
  cat $O/bench_$v.txt
done
timeout -k 5 60 ./tools/probe 1048576 0 > $O/probe_base.txt 2>&1 || exit 1
timeout -k 5 60 ./tools/probe_w512 1048576 0 > $O/probe_w512p.txt 2>&1 || exit 1
grep -A16 "^protect: waves" $O/probe_base.txt $O/probe_w512p.txt
cd /tmp && export TMPDIR=/tmp
C="SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for v in base w512p; do
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$v -o pmc -- $GRAFT_REPO_ROOT/tools/pv_$v 1048576 0 bench > $O/pmc_$v.log 2>&1 || { echo pmc $v failed; tail $O/pmc_$v.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
for v in base w512p; do
  python3 -c "
import csv,glob,collections
f=glob.glob('$O/pmc_$v/**/*counter_collection.csv', recursive=True)[0]
acc=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name'].split('(')[0]
    if 'k_gcm' in k: acc[(k,r['Counter_Name'])].append(float(r['Counter_Value']))
for k in sorted({k for k,_ in acc}):
    g=lambda c: sorted(acc[(k,c)])[len(acc[(k,c)])//2]
    gr=g('GRBM_GUI_ACTIVE')/8; cu=gr*256
    print('$v', k, 'launches', len(acc[(k,'GRBM_GUI_ACTIVE')]), 'cycles/XCD %.4g' % gr, 'LDS busy %.3f' % (g('SQ_LDS_IDX_ACTIVE')/cu),
          'INSTS_LDS %.4g VALU %.4g' % (g('SQ_INSTS_LDS'), g('SQ_INSTS_VALU')),
          'VALU busy(2cyc) %.3f' % (g('SQ_INSTS_VALU')*2/(cu*4)),
          'wave-life/launch %.3f' % (g('SQ_WAVE_CYCLES')*4/(cu*16)),
          'WAIT_INST_LDS/WAVE %.3f WAIT_INST_ANY/WAVE %.3f' % (g('SQ_WAIT_INST_LDS')/g('SQ_WAVE_CYCLES'), g('SQ_WAIT_INST_ANY')/g('SQ_WAVE_CYCLES')),
          'BUSY %.4g' % g('SQ_BUSY_CYCLES'))
"
done
