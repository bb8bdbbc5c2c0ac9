# same-config eager baseline at B 128, and the Llama-1.1B configs (bf16 s2048 B8, bf16 / fp8 s4096 B4, fp8 with
# the hand-written fp8 GEMM)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python benchmarks/eager_baseline.py --batch 128 --attn sdpa > gpurun_out/eager_b128.log 2>&1 || { echo EAGERFAIL; tail -20 gpurun_out/eager_b128.log; exit 1; }
tail -1 gpurun_out/eager_b128.log
timeout -k 10 400 python bench.py --model llama-1.1b --seq 2048 --batch 8 --steps 10 --warmup 3 > gpurun_out/llama_s2048.log 2>&1 || { echo L1FAIL; tail -20 gpurun_out/llama_s2048.log; exit 1; }
tail -1 gpurun_out/llama_s2048.log
timeout -k 10 400 python bench.py --model llama-1.1b --seq 4096 --batch 4 --steps 10 --warmup 3 > gpurun_out/llama_s4096.log 2>&1 || { echo L2FAIL; tail -20 gpurun_out/llama_s4096.log; exit 1; }
tail -1 gpurun_out/llama_s4096.log
timeout -k 10 400 python bench.py --model llama-1.1b --seq 4096 --batch 4 --steps 10 --warmup 3 --precision fp8 > gpurun_out/llama_s4096_fp8.log 2>&1 || { echo L3FAIL; tail -20 gpurun_out/llama_s4096_fp8.log; exit 1; }
tail -1 gpurun_out/llama_s4096_fp8.log
BPE_FP8_GEMM=hip timeout -k 10 400 python bench.py --model llama-1.1b --seq 4096 --batch 4 --steps 10 --warmup 3 --precision fp8 > gpurun_out/llama_s4096_fp8_hip.log 2>&1 || { echo L4FAIL; tail -20 gpurun_out/llama_s4096_fp8_hip.log; exit 1; }
tail -1 gpurun_out/llama_s4096_fp8_hip.log
