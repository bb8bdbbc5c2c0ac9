#!/bin/bash
# fp8 SwiGLU + two-layout cast fusion: tests, then the fp8 Llama config alternating fused / two-pass.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "fp8 or swiglu" 2>&1 | tail -3 || exit 1
for arm in fused twopass fused twopass; do
  echo "== $arm"
  if [ $arm = fused ]; then set_arg=True; else set_arg=False; fi
  timeout -k 10 300 python -u benchmarks/bench_ab.py --set bpe_transformer.models.fused_block._FP8_SWIGLU_CAST=$set_arg \
    -- --model llama-1.1b --seq 4096 --precision fp8 --steps 10 --warmup 3 2>&1 | grep -E '^\{"metric' | cut -c1-200 || exit 1
done
