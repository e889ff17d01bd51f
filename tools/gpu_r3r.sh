#!/bin/bash
# r3r: phase probe (workgroup end spread) with and without the GCM tail pool,
# the full pass (tests, smoke, bench, rehearsal, rocprof), then A/B of the
# committed kernel (head) and the tail-pool build (tail) against this tree.
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
timeout -k 10 120 ./tools/probe 1048576 0 > $O/r3r_probe_1mi.txt 2>&1 || { echo probe failed; tail $O/r3r_probe_1mi.txt; exit 1; }
grep -E "protect|ends|span" $O/r3r_probe_1mi.txt | head -12
timeout -k 10 120 ./tools/probe_tail 1048576 0 > $O/r3r_probe_tail_1mi.txt 2>&1 || { echo probe_tail failed; tail $O/r3r_probe_tail_1mi.txt; exit 1; }
grep -E "protect|ends|span" $O/r3r_probe_tail_1mi.txt | head -12
bash tools/gpu_r3.sh r3r || exit 1
NOTEST=1 bash tools/gpu_ab2.sh r3r_ab ns ns 2 4 -- head tail
