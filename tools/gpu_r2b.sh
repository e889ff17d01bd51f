#!/bin/bash
# GPU pass: parity tests, smoke, then the north-star bench and configs 4/5.
set -uo pipefail
TAG=${1:-r2b}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
timeout -k 10 200 python -u bench.py --cpu-seconds 5 > $O/bench_ns.json 2> $O/bench_ns.err || { echo bench failed; tail $O/bench_ns.err; exit 1; }
cat $O/bench_ns.json
for c in 3 4 5; do
  timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 3 --cpu-all-cores 0 > $O/bench_c$c.json 2> $O/bench_c$c.err || { echo "config $c failed"; tail $O/bench_c$c.err; exit 1; }
  cat $O/bench_c$c.json
done
