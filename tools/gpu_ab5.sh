#!/bin/bash
# Same-box interleaved A/B of the in-tree library against variants/<name>/
# builds (tools/build_variant.py), REPS rounds:
#   tools/gpu_ab5.sh TAG "cfg ..." variant ...
set -uo pipefail
TAG=$1; CFGS=$2; shift 2
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for v in base "$@"; do
    if [ "$v" = base ]; then LP=""; else LP="$GRAFT_REPO_ROOT/variants/$v"; fi
    for c in $CFGS; do
      LD_LIBRARY_PATH=$LP timeout -k 10 200 python -u bench.py --config $c --steps ${STEPS:-20} --warmup 5 --cpu-seconds 0 --cpu-all-cores 0 --no-e2e ${XARGS:-} > $O/b_${c}_${v}_$rep.json 2> $O/b_${c}_${v}_$rep.err || { echo "fail $c $v"; tail -5 $O/b_${c}_${v}_$rep.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/b_${c}_${v}_$rep.json').read().strip().split(chr(10))[-1]); print('$c $v $rep', d['value'], d['kernels_ms'], d['status_ok'])"
    done
  done
done
