#!/bin/bash
# Retry a gpurun call only while the infrastructure reports a transient failure (no box / backoff);
# a call that ran (ok or failed) is never repeated.  usage: gpurun_retry.sh <log> <gpurun args...>
log=$1; shift
for attempt in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1
  if grep -q "status=transient\|no box\|backing off" "$log" && ! grep -q "status=ok\|status=fail" "$log"; then
    sleep 90; continue
  fi
  break
done
tail -4 "$log"
