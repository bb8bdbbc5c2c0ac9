#!/bin/bash
# round 5: kernel-trace profiles of the Llama bf16 s2048 B32 and fp8 s4096 B16 steps at HEAD
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for cfg in "llama_bf16_s2048:--model llama-1.1b --seq 2048" "llama_fp8_s4096:--model llama-1.1b --seq 4096 --precision fp8"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  out=gpurun_out/prof_$tag
  rm -rf $out
  timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $out -o prof -- python3 bench.py --steps 3 --warmup 2 $args > gpurun_out/prof_$tag.log 2>&1
  csv=$(find $out -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_summary.py "$csv" --steps 3 --warmup 2 --title "$tag" > gpurun_out/prof_$tag.md
  rm -rf $out
  head -16 gpurun_out/prof_$tag.md
done
