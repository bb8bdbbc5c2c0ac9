# fp8 GEMM with its MFMAs pinned to their ping-pong sections: numerics, op-level A/B against hipBLASLt, and the
# Llama-1.1B fp8 config end to end with each GEMM path (alternating)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "fp8" --timeout 120 --timeout-method thread > gpurun_out/t_fp8pin.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_fp8pin.log; exit 1; }
tail -1 gpurun_out/t_fp8pin.log
timeout -k 10 300 python benchmarks/gemm_fp8_bench.py > gpurun_out/gemm_fp8_pin.log 2>&1 || { tail -20 gpurun_out/gemm_fp8_pin.log; exit 1; }
cat gpurun_out/gemm_fp8_pin.log
for mode in hip lib hip lib; do
  BPE_FP8_GEMM=$mode timeout -k 10 400 python bench.py --model llama-1.1b --seq 4096 --batch 4 --steps 10 --warmup 3 --precision fp8 > gpurun_out/llama_fp8_$mode.log 2>&1 || { tail -20 gpurun_out/llama_fp8_$mode.log; exit 1; }
  echo "$mode: $(tail -1 gpurun_out/llama_fp8_$mode.log | cut -c1-200)"
done
