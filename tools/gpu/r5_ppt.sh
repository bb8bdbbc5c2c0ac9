#!/bin/bash
# dW routes of round 5 (qkv -> pp, LM head -> ppt at GPT-2 B 128; o -> pp, w13 / head -> ppt at Llama 65 536 tokens)
# vs the previous table (tools/gpu/dw_routes_r5_before.json): route tests, then alternating end-to-end runs
set -o pipefail
O=gpurun_out/ppt
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "weight_grad" > $O/test.log 2>&1 || { echo TESTFAIL; tail -30 $O/test.log; exit 1; }
tail -n 1 $O/test.log
run() {  # tag env args...
  local tag=$1 env=$2; shift 2
  env $env timeout -k 10 400 python -u bench.py "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; return 1; }
  tail -n 1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"], d.get("dw_gemm_routes"))' $tag | tee -a $O/summary.log
}
for r in 1 2; do
  run new_gpt2_$r "X=1" --steps 20 --warmup 5 || exit 1
  run old_gpt2_$r "BPE_GEMM_ROUTES=tools/gpu/dw_routes_r5_before.json" --steps 20 --warmup 5 || exit 1
done
for r in 1 2; do
  run new_s2048_$r "X=1" --steps 10 --warmup 3 --model llama-1.1b --seq 2048 || exit 1
  run old_s2048_$r "BPE_GEMM_ROUTES=tools/gpu/dw_routes_r5_before.json" --steps 10 --warmup 3 --model llama-1.1b --seq 2048 || exit 1
done
