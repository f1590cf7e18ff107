#!/bin/bash
# Submit one gpurun call, re-submitting it only while the pool reports no free slot / a transient infrastructure
# failure (exit 3 or status=transient: nothing ran, nothing charged).  A call that ran is never repeated.
#   bash tools/gpurun_q.sh <log> <timeout_s> '<command>'
LOG=$1
TO=$2
CMD=$3
for attempt in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
