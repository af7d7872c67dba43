#!/bin/bash
# Retry a gpurun call while the pool has no free box (gpurun exit 3: nothing ran / nothing
# charged). Any other exit code is final. Usage: scripts/gpurun_retry.sh LOG TIMEOUT SCRIPT
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
exit 3
