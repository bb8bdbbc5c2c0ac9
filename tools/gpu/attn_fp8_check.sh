# fp8 GEMM + forward v4 numerics (short), then the attention PMC / A/B script
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "fp8 or flash or fp32_output or fp32_buffer" --timeout 120 --timeout-method thread > gpurun_out/t_fp8.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_fp8.log; exit 1; }
tail -3 gpurun_out/t_fp8.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --fwd-ab --bwd-ab --iters 10 > gpurun_out/ab2.log 2>&1
cat gpurun_out/ab2.log
timeout -k 10 300 python benchmarks/gemm_fp8_bench.py > gpurun_out/fp8b.log 2>&1
cat gpurun_out/fp8b.log
bash tools/gpu/attn_split_pmc.sh
