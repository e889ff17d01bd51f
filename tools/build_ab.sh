#!/bin/bash
# Build the probe harness against a given git revision of the engine (A/B base):
#   tools/build_ab.sh REV OUT   (uses the working tree's tools/probe.hip)
set -e
REV=$1; OUT=$2
T=$(mktemp -d)
mkdir -p $T/aioquic_amd/csrc $T/include $T/tools
for f in aioquic_amd/csrc/qpp_engine.hip aioquic_amd/csrc/qpp_device.h aioquic_amd/csrc/qpp_chacha.h include/quic_pp.h; do
  git show $REV:$f > $T/$f
done
cp tools/probe.hip $T/tools/
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I $T/include -o $OUT $T/tools/probe.hip
rm -rf $T
