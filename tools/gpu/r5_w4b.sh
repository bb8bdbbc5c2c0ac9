#!/bin/bash
# round 5: w4 GEMM timing diagnostics (variant build) + the fp8 spike probe (saturation traces)
mkdir -p gpurun_out
BPE_HIP_VARIANT=w4diag timeout -k 10 300 python -u benchmarks/gemm_w4_diag.py > gpurun_out/w4_diag.log 2>&1 || exit $?
timeout -k 10 600 python -u benchmarks/fp8_spike_probe.py --margins 1,2,4 --out gpurun_out/fp8_spike_probe.json > gpurun_out/fp8_spike_probe.log 2>&1
