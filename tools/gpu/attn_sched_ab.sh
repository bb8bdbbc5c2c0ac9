# batched operand reads (44) in the split backward kernels: tests, op-level A/B, attention PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash_bwd_split" > gpurun_out/as_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/as_tests.log; exit 1; }
tail -1 gpurun_out/as_tests.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --bwd-ab --bwd-arms 42,42 44,44 42,45 44,45 --rounds 7 > gpurun_out/as_bwd.log 2>&1 || { echo BWDFAIL; tail gpurun_out/as_bwd.log; exit 1; }
grep -v amdgpu.ids gpurun_out/as_bwd.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 8 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms 42,42 44,45 42,45 --rounds 7 > gpurun_out/as_bwd_llama.log 2>&1 || { echo BWDFAIL2; tail gpurun_out/as_bwd_llama.log; exit 1; }
grep -v amdgpu.ids gpurun_out/as_bwd_llama.log
