# fp8 GEMM numerics first (short), then the attention PMC / A/B script
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "fp8" --timeout 120 --timeout-method thread > gpurun_out/t_fp8.log 2>&1 || { echo FP8FAIL; tail -40 gpurun_out/t_fp8.log; }
tail -3 gpurun_out/t_fp8.log
bash tools/gpu/attn_split_pmc.sh
