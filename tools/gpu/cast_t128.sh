#!/bin/bash
# 128 x 128 two-layout fp8 cast with the next tile prefetched: cast tests, op-level bench (default vs t64 variant).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "cast" 2>&1 | tail -2 || exit 1
for v in "" t64; do
  echo "== cast bench variant '${v:-default}'"
  BPE_HIP_VARIANT=$v timeout -k 10 120 python -u benchmarks/cast_bench.py 2>&1 | grep '"cast_t"' || exit 1
done
