# headline bench twice + the three Llama configs, at HEAD defaults
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/ba_gpt2_$i.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/ba_gpt2_$i.log; exit 1; }
  tail -1 gpurun_out/ba_gpt2_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("gpt2", d["value"], d["ms_per_step"])' | tee -a gpurun_out/bench_all.log
done
rm -f gpurun_out/llama_now.log
bash tools/gpu/llama_now.sh && cat gpurun_out/llama_now.log >> gpurun_out/bench_all.log
