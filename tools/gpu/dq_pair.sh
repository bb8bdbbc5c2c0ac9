# paired dQ query blocks: flash tests, stamps, op-level A/B paired vs unpaired (GPT-2, Llama GQA), e2e
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "flash or sdpa" > gpurun_out/t_flash.log 2>&1 || { echo FLASHFAIL; tail -30 gpurun_out/t_flash.log; exit 1; }
tail -1 gpurun_out/t_flash.log
BPE_HIP_VARIANT=stamps timeout -k 10 120 python benchmarks/attn_stamps.py 2>&1 | grep -v amdgpu.ids | head -12
for i in 1 2; do
  timeout -k 10 120 python benchmarks/attn_bench.py --batch 128 --bwd-ab --iters 10 --rounds 5 --bwd-arms split split_unpaired 2>/dev/null
  timeout -k 10 120 python benchmarks/attn_bench.py --batch 32 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --iters 10 --rounds 3 --bwd-arms split split_unpaired 2>/dev/null
done
