#!/bin/bash
# r5ac: GCM 1 Mi wave / workgroup end times (probe build), by XCD
set -uo pipefail
cd $GRAFT_REPO_ROOT
for a in "1048576 0" "1048576 0"; do
  timeout -k 5 60 tools/probe_prb $a | grep -E "us \(event\)|wave starts|wave ends|workgroup ends" || exit 1
done
