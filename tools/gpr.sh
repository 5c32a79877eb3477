#!/bin/bash
# gpurun with retries on transient infrastructure events only (box lost while
# being prepared, no slot free): nothing ran, nothing was charged.  Any run
# that reached the GPU -- pass or fail -- is returned as is.
#   bash tools/gpr.sh <log> <timeout-s> <command...>
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" || [ $rc -eq 3 ]; then
    sleep 60
    continue
  fi
  break
done
grep "status=" "$LOG"
exit $rc
