#!/bin/bash
# Host-side: re-submit a gpurun call that the infrastructure dropped before the command ran
# (box lost while being prepared / taken away / backing off: nothing charged).  A call whose
# command ran is never repeated.  usage: gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient\|stopped responding while being prepared\|taken away by the GPU service\|backing off" "$LOG" && ! grep -q "merged" "$LOG"; then
    sleep 45; continue
  fi
  exit $rc
done
exit $rc
