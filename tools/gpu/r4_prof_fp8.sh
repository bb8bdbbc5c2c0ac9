# step profile at HEAD (GPT-2 default) + fp8 GEMM hand-vs-library at 65536 and 16384 tokens (persistent fp8
# kernel) + the fp8 Llama config end to end with BPE_FP8_GEMM=routes / hip / lib
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/prof_step.sh r4b | head -40
timeout -k 10 300 python benchmarks/gemm_fp8_bench.py --tokens 65536 --rounds 3 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python benchmarks/gemm_fp8_bench.py --tokens 16384 --rounds 3 2>&1 | grep -v amdgpu.ids
for m in lib hip; do
  BPE_FP8_GEMM=$m timeout -k 10 400 python bench.py --model llama-1.1b --seq 4096 --precision fp8 --steps 10 --warmup 3 > gpurun_out/fp8_$m.log 2>&1 || { echo FP8BENCHFAIL; tail -20 gpurun_out/fp8_$m.log; exit 1; }
  echo "fp8 $m $(tail -1 gpurun_out/fp8_$m.log | cut -c1-160)"
done
