# new defaults (42,42 / fwd v6) + the 8-wave DMA variant: attention tests, op-level A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > gpurun_out/ao2_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/ao2_tests.log; exit 1; }
tail -1 gpurun_out/ao2_tests.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --bwd-ab --bwd-arms 42,42 82,82 42,82 82,42 4,4 --rounds 5 > gpurun_out/ao2_bwd.log 2>&1 || { echo BWDFAIL; tail gpurun_out/ao2_bwd.log; exit 1; }
cat gpurun_out/ao2_bwd.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 8 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms 42,42 82,82 --rounds 5 > gpurun_out/ao2_bwd_llama.log 2>&1 || { echo BWDFAIL2; tail gpurun_out/ao2_bwd_llama.log; exit 1; }
cat gpurun_out/ao2_bwd_llama.log
