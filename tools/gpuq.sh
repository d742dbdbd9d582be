#!/bin/bash
# usage: gpuq.sh LOG TIMEOUT CMD...   retries only while gpurun reports no free box/slot (rc 3)
LOG=$1; shift; TO=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  echo "[gpuq] attempt $i rc=$rc" >> $LOG
  [ $rc -eq 3 ] || exit $rc
  sleep 150
done
