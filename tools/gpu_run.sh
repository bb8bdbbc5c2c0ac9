#!/bin/bash
# GPU-box driver: run steps in order; stop at the first step that faults, aborts or times out.
# usage: tools/gpu_run.sh "<name>:<timeout_s>:<command>" ...
# A step exiting 0 or 1 (pytest failures) lets later steps run; anything else stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] timeout=${to}s: $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc"; tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
exit 0
