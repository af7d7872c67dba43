#!/bin/bash
# Retry a gpurun call while the pool has no free box (gpurun exit 3: nothing ran / nothing
# charged). Any other exit code is final. When gpurun says how long to back off ("retry in
# Ns"), wait that long before the next attempt. Usage: scripts/gpurun_retry.sh LOG TIMEOUT CMD...
LOG=$1; TO=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  wait_s=$(grep -o 'retry in [0-9]*s' "$LOG" | tail -1 | grep -o '[0-9]*')
  sleep $(( ${wait_s:-150} + 15 ))
done
exit 3
