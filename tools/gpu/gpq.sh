#!/bin/bash
# Run one remote-GPU call through a launcher; on a transient "no slot / no box" answer (exit 3: nothing ran or was
# charged) wait a minute and ask again.  The launcher is a parameter: GPU_LAUNCHER (default: `gpurun` on PATH), so
# the script is not tied to one machine's install path.
# usage: GPU_LAUNCHER=<launcher> gpq.sh <timeout-seconds> <log> <cmd...>
T=$1; LOG=$2; shift 2
L=${GPU_LAUNCHER:-gpurun}
for i in $(seq 1 ${GPQ_TRIES:-30}); do
  "$L" --timeout "$T" -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then exit $rc; fi
  sleep 60
done
exit $rc
