#!/bin/bash
# Round-6 GPU pass: parity tests, smoke, the driver's default bench command
# (with the traced host-path round trip), optionally a rocprofv3 kernel trace
# of the default bench and every config.
#   gpurun -- bash tools/gpu_r6.sh TAG [all|tests-only|skip-tests] [prof] [sweep] [rehearse8]
set -uo pipefail
TAG=${1:-r6}
MODE=${2:-all}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ "$MODE" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests_$TAG.log; exit 1; }
  tail -1 $O/gpu_tests_$TAG.log
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo smoke failed; cat $O/smoke_$TAG.log; exit 1; }
  tail -1 $O/smoke_$TAG.log
fi
[ "$MODE" = "tests-only" ] && exit 0
timeout -k 10 300 python -u bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo bench failed; tail $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
for a in "${@:3}"; do
  if [ "$a" = "prof" ]; then
    cd /tmp && export TMPDIR=/tmp
    P=$O/prof_$TAG
    mkdir -p $P
    cd $GRAFT_REPO_ROOT
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o kt -- python3 bench.py --cpu-seconds 0 --no-e2e > $P/kt.log 2>&1 || { echo "rocprof failed"; tail $P/kt.log; exit 1; }
    python3 tools/prof_summary.py $P $P/timed_kernel_trace.csv > $P/summary.md && head -12 $P/summary.md
  fi
  if [ "$a" = "sweep" ]; then
    bash tools/gpu_sweep.sh $TAG || exit 1
  fi
  if [ "$a" = "rehearse8" ]; then
    timeout -k 10 400 python -u bench.py --gpus 8 --rehearse --packets 131072 --cpu-seconds 2 --cpu-all-cores 0 --no-e2e > $O/rehearsal8_$TAG.json 2> $O/rehearsal8_$TAG.err || { echo rehearsal failed; tail $O/rehearsal8_$TAG.err; exit 1; }
    tail -c 600 $O/rehearsal8_$TAG.json
  fi
done
echo gpu_r6-done $TAG
