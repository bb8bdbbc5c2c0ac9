# fp8 weight gradients: kernel tests, wgrad GEMM arms, fp8 Llama end to end (library dW / hand split-K dW /
# bf16 dW), fp8 parity
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "fp8" > gpurun_out/t_fp8.log 2>&1 || { echo FP8TESTFAIL; tail -30 gpurun_out/t_fp8.log; exit 1; }
tail -1 gpurun_out/t_fp8.log
timeout -k 10 300 python benchmarks/gemm_fp8_bench.py --wgrad 2>&1 | grep -v amdgpu.ids
B="--model llama-1.1b --seq 4096 --precision fp8 --steps 10 --warmup 3"
for i in 1 2; do
  timeout -k 10 400 python bench.py $B > gpurun_out/fp8w.log 2>&1 || { echo FP8BENCHFAIL; tail -20 gpurun_out/fp8w.log; exit 1; }
  echo "fp8 wgrad lib  $(tail -1 gpurun_out/fp8w.log | cut -c1-170)"
  timeout -k 10 400 python benchmarks/bench_ab.py --set bpe_transformer.ops.fp8._WGRAD_HIP=True -- $B > gpurun_out/fp8w.log 2>&1 || { echo FP8BENCHFAIL; tail -20 gpurun_out/fp8w.log; exit 1; }
  echo "fp8 wgrad hip  $(tail -1 gpurun_out/fp8w.log | cut -c1-170)"
done
