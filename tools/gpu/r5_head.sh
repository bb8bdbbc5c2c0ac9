#!/bin/bash
# LM-head forward / input-gradient routes: hipBLASLt (tuned table) vs the hand ping-pong kernel
set -o pipefail
O=gpurun_out/head
mkdir -p $O
timeout -k 10 300 python -u benchmarks/head_routes.py > $O/routes.log 2>&1 || { echo FAIL; tail -20 $O/routes.log; exit 1; }
grep -v amdgpu.ids $O/routes.log
