#!/bin/bash
# re-A/B of the bf16 SwiGLU-forward GEMM fusion at d 2048 (Llama-1.1B s2048 B32): BPE_FUSE_SWIGLU_FWD_MAX_D=2048 vs
# the default cap 1024, alternating
set -o pipefail
O=gpurun_out/swfwd
mkdir -p $O
run() {  # tag env args...
  local tag=$1 env=$2; shift 2
  env $env timeout -k 10 400 python -u bench.py "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; return 1; }
  tail -n 1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"])' $tag | tee -a $O/summary.log
}
for r in 1 2; do
  run fused_s2048_$r "BPE_FUSE_SWIGLU_FWD_MAX_D=2048" --steps 10 --warmup 3 --model llama-1.1b --seq 2048 || exit 1
  run cap_s2048_$r "X=1" --steps 10 --warmup 3 --model llama-1.1b --seq 2048 || exit 1
done
