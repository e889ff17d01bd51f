#!/bin/bash
# Build libquicpp.so as of git revision REV into variants/NAME/ (same-box A/B
# of a committed kernel against the working tree; tools/ab_lib.sh runs them).
#   tools/build_rev_variant.sh REV NAME
set -euo pipefail
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" aioquic_amd/csrc include | tar -x -C "$T"
mkdir -p "$ROOT/variants/$NAME"
for u in qpp_engine qpp_plan; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I "$T/include" -c -o "$T/$u.o" "$T/aioquic_amd/csrc/$u.hip" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/variants/$NAME/libquicpp.so" "$T/qpp_engine.o" "$T/qpp_plan.o"
rm -rf "$T"
echo "$ROOT/variants/$NAME/libquicpp.so"
