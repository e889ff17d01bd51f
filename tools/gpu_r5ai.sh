#!/bin/bash
# r5ai: ChaCha20-Poly1305 64 Ki wave / workgroup ends by XCD (probe build)
set -uo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 5 60 tools/probe_prb 65536 2 | grep -E "us \(event\)|wave starts|wave ends|workgroup ends" || exit 1
