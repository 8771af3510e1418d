#!/bin/bash
# gpurun with retries on infrastructure-side failures only (status=transient: no box, box lost while
# being prepared); a command that ran and failed is never retried.
#   tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  grep -q "status=transient" "$LOG" || exit $rc
  grep -q "backing off" "$LOG" && sleep 30 || sleep 60
done
exit $rc
