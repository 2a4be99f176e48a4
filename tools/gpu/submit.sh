#!/bin/bash
# Submit one gpurun call; when the pool has no box or slot free (gpurun exit
# 3: nothing ran, nothing charged) wait and submit it again, up to 12 times.
# Any other outcome (a run that happened, pass or fail) is returned as is.
# usage: tools/gpu/submit.sh TIMEOUT_S 'command'
t=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 75
done
exit 3
