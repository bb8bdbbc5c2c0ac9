# 128-row tiles with (48) and without (47) the batched operand reads: tests + op-level A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash_bwd_split" > gpurun_out/s128_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/s128_tests.log; exit 1; }
tail -1 gpurun_out/s128_tests.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --bwd-ab --bwd-arms 48,48 47,47 48,47 47,48 --rounds 7 2>&1 | grep shape | tee gpurun_out/s128_ab.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 32 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms 48,48 47,47 48,47 --rounds 5 2>&1 | grep shape | tee -a gpurun_out/s128_ab.log
