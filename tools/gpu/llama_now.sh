# Llama-1.1B numbers at HEAD (default micro-batches: 65536 tokens per GPU), bf16 s2048 / s4096 and fp8 s4096
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "--seq 2048" "--seq 4096" "--seq 4096 --precision fp8"; do
  timeout -k 10 400 python -u bench.py --model llama-1.1b $cfg --steps 10 --warmup 3 > gpurun_out/llama_now.tmp 2>&1 || { echo "FAIL $cfg"; tail -20 gpurun_out/llama_now.tmp; exit 1; }
  echo "[$cfg] $(grep '"metric"' gpurun_out/llama_now.tmp | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["micro_batch_per_gpu"], d.get("peak_mem_gb"))')" | tee -a gpurun_out/llama_now.log
done
