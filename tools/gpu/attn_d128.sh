#!/bin/bash
# D = 128 attention, training path: forward + backward with RoPE inside the kernels (--mode fused, the D = 128
# default) vs Q / K pre-rotated by rope_qk_ (--mode block), MHA and GQA.
set -o pipefail
mkdir -p gpurun_out
for args in "--batch 4 --seq 2048 --heads 16 --dim 128" "--batch 4 --seq 2048 --heads 32 --kv-heads 8 --dim 128"; do
  for m in fused block; do
    echo "== $args --mode $m"
    timeout -k 10 120 python -u benchmarks/attn_bench.py $args --mode $m --iters 20 || exit 1
  done
done
