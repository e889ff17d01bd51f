#!/bin/bash
# r5aa: ChaCha20-Poly1305 with the chunk stores dropped (study build, wrong
# output: bounds what hiding the store completions could gain) against base
set -uo pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for v in base nostore; do
    for n in 65536 1048576; do
      echo "$v $n $r $(timeout -k 5 60 tools/probe_$v $n 2 bench)" || exit 1
    done
  done
done
timeout -k 5 60 tools/probe_nostore_probe 65536 2 | grep -E "us \(event\)|wave starts|wave ends"
