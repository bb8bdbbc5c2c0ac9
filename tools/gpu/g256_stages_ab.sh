# 256-tile weight-gradient kernel with 5 LDS stages (3 in flight) vs 4: numerics under both, op-level and end to
# end A/B (alternating)
set -o pipefail
cd $GRAFT_REPO_ROOT
BPE_G256_STAGES=5 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t_g5.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_g5.log; exit 1; }
tail -1 gpurun_out/t_g5.log
for st in 4 5 4 5; do
  BPE_G256_STAGES=$st timeout -k 10 200 python benchmarks/gemm_dw.py > gpurun_out/g5_dw_$st.log 2>&1 || { tail -20 gpurun_out/g5_dw_$st.log; exit 1; }
  echo "stages $st: $(tail -1 gpurun_out/g5_dw_$st.log)"
done
for st in 4 5 4 5; do
  BPE_G256_STAGES=$st timeout -k 10 300 python bench.py > gpurun_out/g5_bench_$st.log 2>&1 || { tail -20 gpurun_out/g5_bench_$st.log; exit 1; }
  echo "stages $st: $(tail -1 gpurun_out/g5_bench_$st.log | cut -c1-200)"
done
