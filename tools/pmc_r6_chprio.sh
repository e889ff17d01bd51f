#!/bin/bash
# Round 6: config 3 (ChaCha20-Poly1305, 64 Ki) with and without issue priority
# by progress (QPP_CHACHA_PRIO=0/1, tools/pv_base): SQ counters in one --pmc
# pass each, wave-lifetime / launch cycles and VALU busy per variant.
#   gpurun -- bash tools/pmc_r6_chprio.sh TAG
set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for v in 0 1; do
  QPP_CHACHA_PRIO=$v timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$v -o pmc -- $GRAFT_REPO_ROOT/tools/pv_base 65536 2 bench > $O/pmc_$v.log 2>&1 || { echo pmc $v failed; tail $O/pmc_$v.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
for v in 0 1; do
  python3 -c "
import csv,glob,collections
f=glob.glob('$O/pmc_$v/**/*counter_collection.csv', recursive=True)[0]
acc=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name'].split('(')[0]
    if 'k_chacha' in k: acc[(k,r['Counter_Name'])].append(float(r['Counter_Value']))
for k in sorted({k for k,_ in acc}):
    g=lambda c: sorted(acc[(k,c)])[len(acc[(k,c)])//2]
    gr=g('GRBM_GUI_ACTIVE')/8; cu=gr*256
    print('prio=$v', k, 'launches', len(acc[(k,'GRBM_GUI_ACTIVE')]), 'cycles/XCD %.4g' % gr,
          'VALU insts %.4g' % g('SQ_INSTS_VALU'), 'VALU busy(2cyc) %.3f' % (g('SQ_INSTS_VALU')*2/(cu*4)),
          'ACTIVE_INST_VALU/launch-SIMD-cycles %.3f' % (g('SQ_ACTIVE_INST_VALU')*4/(cu*4*16)),
          'wave-life/launch %.3f' % (g('SQ_WAVE_CYCLES')*4/g('SQ_WAVES')/gr),
          'WAIT_INST_ANY/WAVE %.3f' % (g('SQ_WAIT_INST_ANY')/g('SQ_WAVE_CYCLES')),
          'waves %d' % g('SQ_WAVES'))
"
done | tee $O/pmc_summary.txt
