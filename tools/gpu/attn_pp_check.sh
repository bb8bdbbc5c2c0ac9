# ping-pong dK/dV kernel: flash numerics first, then the backward A/B and a PMC pass
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "flash" --timeout 120 --timeout-method thread > gpurun_out/t_pp.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_pp.log; exit 1; }
tail -2 gpurun_out/t_pp.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --bwd-ab --iters 10 > gpurun_out/ab3.log 2>&1
timeout -k 10 300 python benchmarks/attn_bench.py --batch 8 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --fwd-ab --iters 10 >> gpurun_out/ab3.log 2>&1
cat gpurun_out/ab3.log
bash tools/gpu/attn_split_pmc.sh > /dev/null 2>&1; grep -E "^## |derived" gpurun_out/attn_pmc/summary.txt
