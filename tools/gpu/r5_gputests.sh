#!/bin/bash
# round 5: the whole GPU suite on the current tree, then the dq16 prologue stamps
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -n 30 gpurun_out/gpu_suite.log; exit 1; }
tail -n 3 gpurun_out/gpu_suite.log
BPE_HIP_VARIANT=stamps timeout -k 10 120 python3 benchmarks/attn_stamps.py --dq-form 1 > gpurun_out/attn_stamps_f1_prologue.log 2>&1 || exit $?
head -3 gpurun_out/attn_stamps_f1_prologue.log
