set -uo pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for c in 2 3; do
for e in 1 10; do
  timeout -k 10 120 python bench.py --config $c --steps 30 --warmup 10 --cpu-seconds 0 --no-e2e --event-every $e > gpurun_out/ev_${c}_${e}.json 2>/dev/null || { echo fail; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ev_${c}_${e}.json'));print('c$c every $e', d['value'], d['ms_per_step'], d['kernels_ms'])"
done; done; done
