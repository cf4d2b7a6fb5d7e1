#!/bin/bash
# Run one gpurun call, waiting for a box: re-submits only when gpurun reports no free box
# (exit 3 / status transient: nothing ran, nothing charged); any other outcome is final.
# Usage: scripts/gpurun_wait.sh TIMEOUT 'command'
T=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  if [ "$rc" != 3 ] && [ "$st" != transient ]; then exit $rc; fi
  sleep 90
done
exit 3
