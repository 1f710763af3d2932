#!/bin/bash
# usage: tools/gpurun_wait.sh LOG TIMEOUT CMD  -- runs CMD through gpurun, retrying only while no
# box is free (exit 3: nothing ran, nothing charged); the log ends with "done"
LOG=$1; T=$2; shift 2
for k in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "no free box right now" $LOG; then break; fi
  sleep 150
done
echo "gpurun rc=$rc" >> $LOG
echo done >> $LOG
