# split attention backward: GPU numerics (flash tests), same-process A/B of the backward forms, then the GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "flash" --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --bwd-ab --iters 10 > gpurun_out/ab1.log 2>&1
timeout -k 10 300 python benchmarks/attn_bench.py --batch 8 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --iters 10 >> gpurun_out/ab1.log 2>&1
cat gpurun_out/ab1.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t2.log 2>&1 || { echo SUITEFAIL; tail -40 gpurun_out/t2.log; exit 1; }
tail -3 gpurun_out/t2.log
