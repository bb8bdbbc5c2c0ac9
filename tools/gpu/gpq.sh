#!/bin/bash
# run a gpurun call; on a transient "no slot / no box" answer (exit 3, nothing ran or charged) wait and ask again
# usage: gpq.sh <timeout> <log> <cmd>
T=$1; LOG=$2; shift 2
for i in $(seq 1 ${GPQ_TRIES:-30}); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $LOG; then exit $rc; fi
  sleep 60
done
exit $rc
