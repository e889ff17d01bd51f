#!/bin/bash
# Re-submit a gpurun call only when the pool reports a transient infrastructure
# failure (box not prepared / backing off: nothing ran, nothing charged).
# Any other outcome -- including a failing command -- is returned as is.
# Usage: tools/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for try in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('/root/repo/gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ] && [ "$rc" != "3" ]; then exit $rc; fi
  echo "[retry] transient pool failure (try $try), waiting" >&2
  sleep 60
done
exit 3
