#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool has no free box / slot (the
# call then never ran and nothing was charged: gpurun exit 3 or a "transient" status);
# any call that ran -- pass or fail -- ends this script.  Usage:
#   tools/gpu/queue.sh LOG TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then
    echo "[queue] attempt $i: no box, waiting" >> "$log.queue"
    sleep 120
    continue
  fi
  exit $rc
done
exit 3
