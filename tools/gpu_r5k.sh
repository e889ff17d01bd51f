#!/bin/bash
# r5k: copy-submission probe; ChaCha20-Poly1305 select-free whole-chunk step
# (variants/chwhole) against the tree, config 3 at 64 Ki and 1 Mi, interleaved
set -uo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/memcpy_submit_probe.py > gpurun_out/memcpy_submit_probe.json 2>&1 || { echo submit probe failed; tail -5 gpurun_out/memcpy_submit_probe.json; }
tail -1 gpurun_out/memcpy_submit_probe.json
bash tools/gpu_ab5.sh r5k_c3 3 chwhole
XARGS="--packets 1048576" bash tools/gpu_ab5.sh r5k_c3m 3 chwhole
