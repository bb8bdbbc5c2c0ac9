#!/bin/bash
# kernel-trace profile of the Llama fp8 s4096 B16 step at HEAD (coalesced fp8 casts, auto dQ form)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag=llama_fp8_s4096
out=gpurun_out/prof_$tag
rm -rf $out
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $out -o prof -- python3 bench.py --steps 3 --warmup 2 --model llama-1.1b --seq 4096 --precision fp8 > gpurun_out/prof_$tag.log 2>&1
csv=$(find $out -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$csv" --steps 3 --warmup 2 --title "$tag" > gpurun_out/prof_$tag.md
rm -rf $out
head -30 gpurun_out/prof_$tag.md
