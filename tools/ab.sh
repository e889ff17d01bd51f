#!/bin/bash
# A/B of kernel switches on the bench workload (GPU box): one line per variant.
set -uo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --config ${CFG:-2} --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab_$name.json 2>/dev/null || { echo "fail $name"; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$name.json')); print('$name', d['value'], d['kernels_ms'], d['status_ok'])"
}
for v in "$@"; do
  IFS=, read -ra kv <<< "$v"
  run "${v//[=,]/_}" "${kv[@]}" || exit 1
done
