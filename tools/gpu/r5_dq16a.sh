#!/bin/bash
# round 5: the 16-queries-per-wave dQ kernel (tests, op-level A/B), the fp8 cross / same-weights checks, the LDS-DMA
# issue microbenchmark
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "dq16 or split_vs_fused" --timeout 120 --timeout-method thread > gpurun_out/dq16_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/attn_bench.py --batch 128 --bwd-ab --bwd-arms split split_dq16 --rounds 5 > gpurun_out/dq16_ab_gpt2.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/attn_bench.py --batch 32 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms split split_dq16 --rounds 5 > gpurun_out/dq16_ab_llama.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/fp8_spike_probe.py --cross 18,25,73 --out gpurun_out/fp8_cross.json > gpurun_out/fp8_cross.log 2>&1 || exit $?
BPE_PARITY_LOG=gpurun_out/parity timeout -k 10 300 python -u -m pytest tests/test_training_parity_gpu.py -x -q -k same_weights --timeout 240 --timeout-method thread > gpurun_out/fp8_same_weights_test.log 2>&1 || exit $?
timeout -k 10 120 ./benchmarks/dma_issue_bench.bin > gpurun_out/dma_issue_bench.log 2>&1
