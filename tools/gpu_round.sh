#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench (with CPU baseline + e2e), rocprof.
# Usage (via gpurun): bash tools/gpu_round.sh TAG
set -uo pipefail
TAG=${1:-r1}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests_$TAG.log; exit 1; }
tail -3 $O/gpu_tests_$TAG.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo smoke failed; cat $O/smoke_$TAG.log; exit 1; }
cat $O/smoke_$TAG.log
timeout -k 10 200 python -u bench.py --e2e --check > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo bench failed; tail $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
bash tools/profile.sh $TAG || { echo profile failed; exit 1; }
