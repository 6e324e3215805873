#!/bin/bash
# Submit a gpurun command, waiting and resubmitting only while gpurun reports "no box or slot free"
# (exit 3: nothing ran, nothing charged).  Any other exit code -- including a failing GPU step --
# is returned as is.  $1 = gpurun --timeout seconds, $2 = command, $3 = log file.
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2" > "$3" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 75
done
exit 3
