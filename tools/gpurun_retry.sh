#!/bin/bash
# Submit a gpurun command, waiting and resubmitting only while gpurun reports that nothing ran:
# "no box or slot free" (exit 3) or a transient infrastructure event (status=transient: the box was
# withdrawn before the command ran; not charged).  Any other outcome -- including a failing GPU
# step -- is returned as is.  $1 = gpurun --timeout seconds, $2 = command, $3 = log file.
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2" > "$3" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$3"; then exit $rc; fi
  sleep 75
done
exit 3
