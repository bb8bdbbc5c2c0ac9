# persistent gemm_pp + QKV/RoPE epilogue end to end: GEMM tests, GEMM A/B incl. the input-gradient shapes, then
# the headline bench alternating: default (persistent + fused QKV RoPE), one-tile variant build
# (BPE_HIP_VARIANT=tile), unfused QKV RoPE (module flag), twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or swiglu or fp8 or rope" > gpurun_out/t_gemm.log 2>&1 || { echo GEMMFAIL; tail -30 gpurun_out/t_gemm.log; exit 1; }
tail -1 gpurun_out/t_gemm.log
timeout -k 10 300 python benchmarks/gemm_persist_ab.py --model gpt2 --rounds 3 2>&1 | grep -v amdgpu.ids
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/pe_bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/pe_bench.log; exit 1; }
  echo "default      $(tail -1 gpurun_out/pe_bench.log | cut -c1-150)"
  BPE_HIP_VARIANT=tile timeout -k 10 300 python bench.py > gpurun_out/pe_bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/pe_bench.log; exit 1; }
  echo "one-tile     $(tail -1 gpurun_out/pe_bench.log | cut -c1-150)"
  timeout -k 10 300 python benchmarks/bench_ab.py --set bpe_transformer.models.fused_block._FUSE_QKV_ROPE=False > gpurun_out/pe_bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/pe_bench.log; exit 1; }
  echo "unfused-rope $(tail -1 gpurun_out/pe_bench.log | cut -c1-150)"
done
