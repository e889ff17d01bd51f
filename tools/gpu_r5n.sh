#!/bin/bash
# Round-5 GPU pass: parity tests, smoke, the driver's default bench command,
# an 8-rank rehearsal of bench.py --gpus 8 on the one-GPU box, and a
# rocprofv3 kernel trace of the default bench (timed launches summarised).
#   gpurun -- bash tools/gpu_r5.sh TAG [skip-tests|tests-only]
set -uo pipefail
TAG=${1:-r5}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests_$TAG.log; exit 1; }
  tail -1 $O/gpu_tests_$TAG.log
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo smoke failed; cat $O/smoke_$TAG.log; exit 1; }
  tail -1 $O/smoke_$TAG.log
fi
[ "${2:-}" = "tests-only" ] && exit 0
timeout -k 10 300 python -u bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo bench failed; tail $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
timeout -k 10 400 python -u bench.py --gpus 8 --rehearse --packets 131072 --cpu-seconds 2 --cpu-all-cores 0 --no-e2e > $O/rehearsal8_$TAG.json 2> $O/rehearsal8_$TAG.err || { echo rehearsal failed; tail $O/rehearsal8_$TAG.err; exit 1; }
tail -c 400 $O/rehearsal8_$TAG.json
cd /tmp && export TMPDIR=/tmp
P=$O/prof_$TAG
mkdir -p $P
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o kt -- python3 bench.py --cpu-seconds 0 --no-e2e > $P/kt.log 2>&1 || { echo "rocprof failed"; tail $P/kt.log; exit 1; }
python3 tools/prof_summary.py $P $P/timed_kernel_trace.csv > $P/summary.md && head -12 $P/summary.md
echo gpu_r5-done $TAG
bash tools/gpu_sweep.sh $TAG
