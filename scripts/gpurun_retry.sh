#!/bin/bash
# gpurun, retried only while the pool has no free box / slot (exit 3 or a 'transient' verdict
# with nothing run); any other outcome is returned as is.  usage: scripts/gpurun_retry.sh TIMEOUT 'cmd'
T=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json; d=json.load(open('gpurun_out/.last_call.json')); print(d['status'], d.get('run_s', 0))" 2>/dev/null)
  if [ $rc -eq 3 ] || [[ "$st" == transient* ]]; then echo "[retry $i: $st]"; sleep 90; continue; fi
  exit $rc
done
exit $rc
