# same-box end to end: round-3 end tree (old_r3/, commit 0797fe2, its own build) vs HEAD, alternating:
# GPT-2 B 128 and Llama-1.1B s2048 B32 bf16
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L="--model llama-1.1b --seq 2048 --steps 10 --warmup 3"
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/ab.log 2>&1 || { echo FAIL; tail -20 gpurun_out/ab.log; exit 1; }
  echo "r4 gpt2  $(tail -1 gpurun_out/ab.log | cut -c1-130)"
  (cd old_r3 && timeout -k 10 300 python bench.py > ../gpurun_out/ab.log 2>&1) || { echo FAIL; tail -20 gpurun_out/ab.log; exit 1; }
  echo "r3 gpt2  $(tail -1 gpurun_out/ab.log | cut -c1-130)"
  timeout -k 10 400 python bench.py $L > gpurun_out/ab.log 2>&1 || { echo FAIL; tail -20 gpurun_out/ab.log; exit 1; }
  echo "r4 llama $(tail -1 gpurun_out/ab.log | cut -c1-130)"
  (cd old_r3 && timeout -k 10 400 python bench.py $L > ../gpurun_out/ab.log 2>&1) || { echo FAIL; tail -20 gpurun_out/ab.log; exit 1; }
  echo "r3 llama $(tail -1 gpurun_out/ab.log | cut -c1-130)"
done
