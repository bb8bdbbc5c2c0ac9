#!/bin/bash
# 128 x 128 two-layout fp8 casts (plain and SwiGLU-fused): tests, cast bench, fp8 Llama config twice.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "cast or fp8 or swiglu" 2>&1 | tail -2 || exit 1
timeout -k 10 120 python -u benchmarks/cast_bench.py 2>&1 | grep '"cast_t"' || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model llama-1.1b --seq 4096 --precision fp8 --steps 10 --warmup 3 2>&1 \
    | grep -E '^\{"metric' | cut -c1-200 || exit 1
done
