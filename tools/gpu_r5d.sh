#!/bin/bash
# r5d: config 4 (and the north star) of this tree against the final round-3
# tree (variants/r3zf_tree: git archive 1d41bb1, built in place), same box,
# interleaved, every timed step event-bracketed in both.
set -uo pipefail
TAG=${1:-r5d}
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
for rep in 1 2 3; do
  for v in head r3zf; do
    for c in ${CFGS:-4 ns}; do
      if [ $v = head ]; then D=$GRAFT_REPO_ROOT; X="--no-e2e"; else D=$GRAFT_REPO_ROOT/variants/r3zf_tree; X=""; fi
      (cd $D && timeout -k 10 200 python -u bench.py --config $c --steps 20 --warmup 5 --cpu-seconds 0 --cpu-all-cores 0 --event-every 1 $X) > $O/b_${c}_${v}_$rep.json 2> $O/b_${c}_${v}_$rep.err || { echo "fail $c $v"; tail -5 $O/b_${c}_${v}_$rep.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/b_${c}_${v}_$rep.json').read().strip().split(chr(10))[-1]); print('$c $v $rep', d['value'], d['kernels_ms'], d['status_ok'])"
    done
  done
done
