#!/bin/bash
# Build bench-mode probe binaries (tools/probe.hip without QPP_PROBE) for A/B
# studies: tools/build_probe_variants.sh name1 "-DFLAG=1 ..." name2 "..." ...
# -> tools/pv_<name> (git-ignored; travels to the GPU box).  "base" = no flags.
set -euo pipefail
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include $flags -c -o /tmp/pv_$name.o tools/probe.hip 2>&1 | grep -v warning || true
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -o tools/pv_$name /tmp/pv_$name.o build/obj/qpp_plan.o build/obj/qpp_source_hash.o
  echo built tools/pv_$name
done
