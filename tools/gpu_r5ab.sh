#!/bin/bash
# r5ab: ChaCha20-Poly1305 with the next step's LDS-DMA issued before this
# step's stores (QPP_CH_EARLYDMA: the step waits for its input, not for the
# previous stores' completion) against base; correctness pass then timing
set -uo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 5 60 tools/probe_early 65536 2 | grep -E "status|diffs|bad" || exit 1
timeout -k 5 60 tools/probe_early 1048573 2 | grep -E "status|bad" || exit 1
for r in 1 2 3; do
  for v in base early; do
    for n in 65536 1048576; do
      echo "$v $n $r $(timeout -k 5 60 tools/probe_$v $n 2 bench)" || exit 1
    done
  done
done
