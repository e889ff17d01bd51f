#!/bin/bash
# Timing-only A/B (no: ablation variants compute wrong bytes) of the
# in-tree library against variants/<name>/ builds: tools/gpu_abl.sh cfg packets variant...
set -uo pipefail
CFG=$1; PK=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/abl
mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in base "$@"; do
  if [ "$v" = base ]; then LP=""; else LP="$GRAFT_REPO_ROOT/variants/$v"; fi
  LD_LIBRARY_PATH=$LP timeout -k 10 150 python -u bench.py --config $CFG --packets $PK --steps ${STEPS:-10} --warmup 3 --cpu-seconds 0 --cpu-all-cores 0 > $O/b_$v.json 2> $O/b_$v.err || { echo "fail $v"; tail -5 $O/b_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().split(chr(10))[-1]); print('$v', d['value'], d['kernels_ms'])"
done
