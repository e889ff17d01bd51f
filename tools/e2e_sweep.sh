#!/bin/bash
# End-to-end (pinned host -> H2D -> protect -> unprotect -> D2H) sweep at 1Mi packets.
# Usage (via gpurun): bash tools/e2e_sweep.sh TAG
set -uo pipefail
TAG=${1:-e2e}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for sc in "per-chunk 4 16" "staged 3 8" "staged 3 16" "staged 3 32" "staged 3 64"; do set -- $sc
  f=gpurun_out/${TAG}_$1_$3.json
  timeout -k 10 200 python -u bench.py --packets 1048576 --steps 5 --warmup 2 --cpu-seconds 0 --e2e \
    --e2e-mode $1 --e2e-streams $2 --e2e-chunks $3 > $f 2>gpurun_out/${TAG}.err || { tail gpurun_out/${TAG}.err; exit 1; }
  python -c "import json; d=json.load(open('$f')); print('$1 $3', d['e2e'])"
done
