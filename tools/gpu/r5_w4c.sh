#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_w4_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w4_test2.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/gemm_w4_bench.py --model gpt2 --square 8192 > gpurun_out/w4_bench_gpt2_r.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/gemm_w4_bench.py --model llama --tokens 65536 > gpurun_out/w4_bench_llama_r.log 2>&1 || exit $?
BPE_HIP_VARIANT=w4diag timeout -k 10 300 python -u benchmarks/gemm_w4_diag.py > gpurun_out/w4_diag2.log 2>&1
