#!/bin/bash
# r5o: the default bench line three times (host-path leg first, on a freed state)
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5o; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --cpu-seconds 0 --cpu-all-cores 0 > $O/b$r.json 2> $O/b$r.err || { echo bench failed; tail $O/b$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b$r.json').read().strip().split(chr(10))[-1]); print(d['value'], d['e2e']['gib_s'], d['e2e_host_devices'])"
done
