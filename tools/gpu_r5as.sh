#!/bin/bash
# r5as: host copy bandwidth on the GPU box's host, memcpy against
# non-temporal stores (CPU only), 6 and 16 threads
set -uo pipefail
cd $GRAFT_REPO_ROOT
for t in 6 16; do timeout -k 5 120 tools/ntbench $t || exit 1; done
