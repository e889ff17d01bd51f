#!/bin/bash
# r5w: wave start / end distribution of the packet kernels (probe build):
# ChaCha20-Poly1305 and AES-128-GCM at 64 Ki and 1 Mi
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5w; mkdir -p $O
for a in "65536 2" "1048576 2" "65536 0"; do
  timeout -k 5 60 tools/probe_chacha $a > $O/p_${a// /_}.txt 2>&1 || { echo "probe $a failed"; tail $O/p_${a// /_}.txt; exit 1; }
  echo "== $a"; grep -E "us \(event\)|waves|wave starts|wave ends|workgroup ends" $O/p_${a// /_}.txt
done
