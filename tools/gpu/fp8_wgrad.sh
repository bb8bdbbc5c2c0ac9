# fp8 weight gradients: kernel tests, wgrad GEMM fp8 vs bf16 route, fp8 Llama end to end with / without fp8 dW,
# and the fp8 parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "fp8" > gpurun_out/t_fp8.log 2>&1 || { echo FP8TESTFAIL; tail -30 gpurun_out/t_fp8.log; exit 1; }
tail -1 gpurun_out/t_fp8.log
timeout -k 10 300 python benchmarks/gemm_fp8_bench.py --wgrad 2>&1 | grep -v amdgpu.ids
for i in 1 2; do
  timeout -k 10 400 python bench.py --model llama-1.1b --seq 4096 --precision fp8 --steps 10 --warmup 3 > gpurun_out/fp8w.log 2>&1 || { echo FP8BENCHFAIL; tail -20 gpurun_out/fp8w.log; exit 1; }
  echo "fp8 wgrad   $(tail -1 gpurun_out/fp8w.log | cut -c1-170)"
  timeout -k 10 400 python benchmarks/bench_ab.py --set bpe_transformer.models.transformer.FP8_WGRAD=False -- --model llama-1.1b --seq 4096 --precision fp8 --steps 10 --warmup 3 > gpurun_out/fp8w.log 2>&1 || { echo FP8BENCHFAIL; tail -20 gpurun_out/fp8w.log; exit 1; }
  echo "bf16 wgrad  $(tail -1 gpurun_out/fp8w.log | cut -c1-170)"
done
BPE_PARITY_LOG=gpurun_out/parity timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/test_training_parity_gpu.py -k fp8 > gpurun_out/t_fp8par.log 2>&1 || { echo PARFAIL; tail -30 gpurun_out/t_fp8par.log; exit 1; }
tail -1 gpurun_out/t_fp8par.log
