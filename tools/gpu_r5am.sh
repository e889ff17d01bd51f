#!/bin/bash
# r5am: GCM 1 Mi phase breakdown per wave (probe build), protect and unprotect
set -uo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 5 60 tools/probe_prb 1048576 0 | grep -vE "res\[|pkt [0-9]" || exit 1
