#!/bin/bash
# One GPU-box pass: parity tests, smoke, default bench (+ e2e), every config,
# rocprof for configs 2 and 3.   Usage (via gpurun): bash tools/gpu_round.sh TAG
set -uo pipefail
TAG=${1:-r1}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests_$TAG.log; exit 1; }
tail -1 $O/gpu_tests_$TAG.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo smoke failed; cat $O/smoke_$TAG.log; exit 1; }
tail -1 $O/smoke_$TAG.log
timeout -k 10 300 python -u bench.py --e2e > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo bench failed; tail $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
for c in 3 4 5; do
  timeout -k 10 200 python -u bench.py --config $c --cpu-seconds 3 --cpu-all-cores 0 > $O/sweep_${TAG}_c$c.json 2>$O/sweep_${TAG}_c$c.err || { echo "config $c failed"; tail $O/sweep_${TAG}_c$c.err; exit 1; }
done
timeout -k 10 200 python -u bench.py --config 2 --packets 1048576 --cpu-seconds 0 > $O/sweep_${TAG}_1mi.json 2>$O/sweep_${TAG}_1mi.err || { echo "1mi failed"; exit 1; }
timeout -k 10 200 python -u bench.py --config 3 --packets 1048576 --cpu-seconds 0 > $O/sweep_${TAG}_c3_1mi.json 2>$O/sweep_${TAG}_c3_1mi.err || { echo "c3 1mi failed"; exit 1; }
bash tools/profile.sh ${TAG}_c2 && bash tools/profile.sh ${TAG}_c3 --config 3 --steps 5 --warmup 2 --cpu-seconds 0 || { echo profile failed; exit 1; }
