#!/bin/bash
# round-5 end: same-box A/B of HEAD against the round-4 tree (ab_r4/ = git c9ddb60 with its own in-tree library),
# alternating: GPT-2 B 128 (3 pairs) and the Llama fp8 s4096 B16 config (2 pairs)
set -o pipefail
mkdir -p gpurun_out/r4ab2
O=gpurun_out/r4ab2
run() {  # tree tag args...
  local tree=$1 tag=$2; shift 2
  (cd $tree && timeout -k 10 400 python -u bench.py "$@") > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; return 1; }
  tail -n 1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"])' $tag | tee -a $O/summary.log
}
for r in 1 2 3; do
  run . head_gpt2_$r --steps 20 --warmup 5 || exit 1
  run ab_r4 r4_gpt2_$r --steps 20 --warmup 5 || exit 1
done
for r in 1 2; do
  run . head_fp8_$r --steps 10 --warmup 3 --model llama-1.1b --seq 4096 --precision fp8 || exit 1
  run ab_r4 r4_fp8_$r --steps 10 --warmup 3 --model llama-1.1b --seq 4096 --precision fp8 || exit 1
done
