#!/bin/bash
# Same-box interleaved A/B of one environment switch on bench configs:
#   tools/gpu_env_ab.sh TAG "ENV=1" cfg...   (base = switch unset)
set -uo pipefail
TAG=$1; ENVSW=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for c in "$@"; do
  for rep in 1 2 3; do
    for v in base var; do
      if [ $v = base ]; then E=""; else E="$ENVSW"; fi
      env $E timeout -k 10 150 python -u bench.py --config $c --packets ${PKTS:-0} --steps ${STEPS:-20} --warmup 5 --cpu-seconds 0 --cpu-all-cores 0 > $O/b_${c}_${v}_$rep.json 2> $O/b_${c}_${v}_$rep.err || { echo "fail $c $v"; tail -5 $O/b_${c}_${v}_$rep.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/b_${c}_${v}_$rep.json').read().strip().split(chr(10))[-1]); print('$c $v', d['value'], d['kernels_ms'], d.get('round_trip_checked'), d['status_ok'])"
    done
  done
done
