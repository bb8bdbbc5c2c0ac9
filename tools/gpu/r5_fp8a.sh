#!/bin/bash
# round 5: fp8 race test + fp8 parity with the gradient margin + the same-weights spike probe
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "fp8 or sdpa or masked" --timeout 300 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/fp8_spike_probe.py --same-weights 18,25,73 --out gpurun_out/fp8_same_weights.json > gpurun_out/fp8_same_weights.log 2>&1 || exit $?
BPE_PARITY_LOG=gpurun_out/parity timeout -k 10 900 python -u -m pytest tests/test_training_parity_gpu.py -x -q -k fp8 --timeout 600 --timeout-method thread > gpurun_out/fp8_parity.log 2>&1
