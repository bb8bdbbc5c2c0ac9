# Llama-1.1B s2048 micro-batch sizing: B 8 (tuned table, and library heuristics), B 16 / 32 (heuristics; dW routes
# timed at first use)
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { tag=$1; shift; timeout -k 10 400 python bench.py --model llama-1.1b --seq 2048 --steps 8 --warmup 3 "$@" > gpurun_out/lb_$tag.log 2>&1 || { tail -20 gpurun_out/lb_$tag.log; exit 1; }; echo "$tag: $(tail -1 gpurun_out/lb_$tag.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["gemm_tuning"])')"; }
run b8 --batch 8
run b8_heur --batch 8 --gemm-tuning off
run b16 --batch 16
run b32 --batch 32
run b8_again --batch 8
for mode in routes lib routes lib; do
  BPE_FP8_GEMM=$mode timeout -k 10 400 python bench.py --model llama-1.1b --seq 4096 --batch 4 --steps 10 --warmup 3 --precision fp8 > gpurun_out/llama_fp8r_$mode.log 2>&1 || { tail -20 gpurun_out/llama_fp8r_$mode.log; exit 1; }
  echo "fp8 $mode: $(tail -1 gpurun_out/llama_fp8r_$mode.log | cut -c1-200)"
done
