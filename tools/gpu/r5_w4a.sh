#!/bin/bash
# round 5: w4 GEMM correctness + op-level A/B vs gemm_pp / hipBLASLt, then the headline bench on the same box
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_w4_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/w4_test.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/gemm_w4_bench.py --model gpt2 --square 8192 > gpurun_out/w4_bench_gpt2.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/gemm_w4_bench.py --model llama --tokens 65536 > gpurun_out/w4_bench_llama.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/bench_base.log 2>&1
