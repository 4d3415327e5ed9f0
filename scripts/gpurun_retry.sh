#!/bin/bash
# Submit one gpurun call, re-submitting only while the pool has no free slot or box (gpurun ran nothing and
# charged nothing: exit 3 / "nothing was charged").  A call that ran -- whatever its outcome -- is never
# repeated.  usage: scripts/gpurun_retry.sh <timeout-s> '<command>'   (tries up to 20 times, 2 min apart)
T=$1
shift
for k in $(seq 1 20); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  echo "$out" | tail -4
  if [ $rc -eq 3 ] || echo "$out" | grep -q "nothing was charged\|no free box\|stopped responding while being prepared"; then
    sleep 120
    continue
  fi
  exit $rc
done
exit 3
