#!/bin/bash
# gpurun wrapper: retries ONLY when no box was obtained (transient / exit 3: nothing ran, nothing charged).
# usage: tools/gpu.sh LOGFILE TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for a in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" $LOG; then sleep 40; continue; fi
  break
done
tail -3 $LOG
exit $rc
