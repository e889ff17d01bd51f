#!/bin/bash
# r5x: ChaCha20 step priority by progress (QPP_CH_PRIO) against the base
# engine, bench mode of the probe harness (event-timed protect + unprotect),
# interleaved, 64 Ki and 1 Mi; then the wave timeline of the variant at 64 Ki
set -uo pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5x; mkdir -p $O
for r in 1 2 3; do
  for v in base chprio; do
    for n in 65536 1048576; do
      echo "$v $n $r $(timeout -k 5 60 tools/probe_$v $n 2 bench)" || exit 1
    done
  done
done
timeout -k 5 60 tools/probe_chprio_probe 65536 2 > $O/timeline_64k.txt 2>&1 && grep -E "us \(event\)|wave starts|wave ends" $O/timeline_64k.txt
# GCM: step priority by progress (QPP_GCM_PRIO), 64 Ki (config 2) and 1 Mi
for r in 1 2 3; do
  for v in base gcmprio; do
    for n in 65536 1048576; do
      echo "$v gcm $n $r $(timeout -k 5 60 tools/probe_$v $n 0 bench)" || exit 1
    done
  done
done
for v in base gcmprio; do
  timeout -k 5 60 tools/probe_${v}_probe 65536 0 > $O/timeline_gcm_${v}.txt 2>&1 && echo "== $v" && grep -E "us \(event\)|wave starts|wave ends" $O/timeline_gcm_${v}.txt
done
