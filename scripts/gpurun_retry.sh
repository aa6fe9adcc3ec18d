#!/bin/bash
# gpurun, re-submitted only when the call never ran (an infrastructure "transient" status or
# exit 3: no box / slot free; nothing charged).  A call that ran is never repeated.
#   scripts/gpurun_retry.sh <log> <timeout_s> '<command>'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 ${RETRIES:-20}); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" || [ $rc -eq 3 ]; then
    echo "[retry $i: infrastructure, nothing ran]" >> "$LOG.retries"
    sleep 120
    continue
  fi
  exit $rc
done
exit 3
