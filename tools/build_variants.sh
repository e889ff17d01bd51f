#!/bin/bash
# Build probe binaries of engine variants (CPU container): tools/probe_<name>
#   tools/build_variants.sh name="-DFLAG=.. ..." ...
set -e
cd "$(dirname "$0")/.."
pids=()
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include $flags -o tools/probe_$name tools/probe.hip > /tmp/build_$name.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
