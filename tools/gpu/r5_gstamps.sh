#!/bin/bash
# per-workgroup phase stamps of the ping-pong GEMMs (both forms) at GPT-2 B 128: where the fused SwiGLU GEMMs' time goes
set -o pipefail
O=gpurun_out/gstamps
mkdir -p $O
BPE_HIP_VARIANT=stamps timeout -k 10 300 python -u benchmarks/gemm_stamps.py > $O/stamps.log 2>&1 || { echo FAIL; tail -20 $O/stamps.log; exit 1; }
grep -v amdgpu.ids $O/stamps.log
