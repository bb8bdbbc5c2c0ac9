#!/bin/bash
# round-5 end: same-box A/B of HEAD against the round-4 tree (ab_r4/ = git c9ddb60, own in-tree library), alternating:
# GPT-2 B 128 and the two Llama bf16 configs, two pairs each
set -o pipefail
mkdir -p gpurun_out/r4ab3
O=gpurun_out/r4ab3
run() {  # tree tag args...
  local tree=$1 tag=$2; shift 2
  (cd $tree && timeout -k 10 400 python -u bench.py "$@") > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; return 1; }
  tail -n 1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"])' $tag | tee -a $O/summary.log
}
for r in 1 2; do
  run . head_gpt2_$r --steps 20 --warmup 5 || exit 1
  run ab_r4 r4_gpt2_$r --steps 20 --warmup 5 || exit 1
done
for cfg in "s2048:--model llama-1.1b --seq 2048" "s4096:--model llama-1.1b --seq 4096"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  for r in 1 2; do
    run . head_llama_${tag}_$r --steps 10 --warmup 3 $args || exit 1
    run ab_r4 r4_llama_${tag}_$r --steps 10 --warmup 3 $args || exit 1
  done
done
