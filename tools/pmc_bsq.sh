#!/bin/bash
# Quad-bitsliced AES-CTR against the T-table form (tools/mb_bsq.hip): wall
# time, then LDS-array and VALU counters per variant (1 workgroup of 1024
# threads per CU, as k_gcm).  LDS busy = SQ_LDS_IDX_ACTIVE per CU-cycle
# (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs); VALU issue share = SQ_INSTS_VALU x 2
# cycles per wave-instruction over the 4 SIMDs' cycles.
#   gpurun -- bash tools/pmc_bsq.sh <tag>
set -uo pipefail
T=${1:-bsq}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/mb_bsq > $O/wall.txt 2>&1 || { echo mb_bsq failed; cat $O/wall.txt; exit 1; }
cat $O/wall.txt
C="SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc -o pmc -- ./tools/mb_bsq > $O/pmc.log 2>&1 || { echo pmc failed; tail $O/pmc.log; exit 1; }
python3 - "$O" <<'EOF'
import csv, glob, collections, sys
o = sys.argv[1]
f = glob.glob(o + '/pmc/*counter_collection.csv')[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0]
    if 'k_run' in k:
        acc[(k, r['Counter_Name'])].append(float(r['Counter_Value']))
blocks = 2048 * 1024 * 32 * 2
for k in sorted({k for k, _ in acc}):
    g = lambda c: sum(acc[(k, c)]) / len(acc[(k, c)])
    cu = g('GRBM_GUI_ACTIVE') / 8 * 256
    print('%-32s LDS busy %.3f  VALU issue %.3f  LDS-cyc/blk %.2f  VALU/blk %.1f  INSTS_LDS/blk %.2f  '
          'WAIT_INST_LDS %.3f  WAIT_INST_ANY %.3f of wave-cycles' % (
              k, g('SQ_LDS_IDX_ACTIVE') / cu, g('SQ_INSTS_VALU') * 2 / (cu * 4),
              g('SQ_LDS_IDX_ACTIVE') / blocks, g('SQ_INSTS_VALU') * 64 / blocks, g('SQ_INSTS_LDS') * 64 / blocks,
              g('SQ_WAIT_INST_LDS') / g('SQ_WAVE_CYCLES'), g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES')))
EOF
