#!/bin/bash
# gpurun, retried (every 3 minutes, at most 10 times) only while no box or slot is free (exit code 3:
# nothing ran, nothing charged).  Any other outcome is final.  Usage: tools/gpurun_retry.sh <log> <timeout> <cmd...>
LOG=$1; TO=$2; shift 2
for i in $(seq 1 10); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $LOG; then exit $rc; fi
  sleep 180
done
exit $rc
