#!/bin/bash
# round 5: the 16-keys-per-wave dK/dV kernel -- tests against the 32-key kernel and the oracle, op-level A/B
mkdir -p gpurun_out/dkv16
O=gpurun_out/dkv16
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "dkv16 or dq16 or flash_bwd_split" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -n 40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 python -u benchmarks/attn_bench.py --batch 128 --bwd-ab --bwd-arms split_dq16 split_dq16_dkv16 --rounds 5 > $O/ab_gpt2.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/attn_bench.py --batch 32 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms split_dq16 split_dq16_dkv16 --rounds 5 > $O/ab_llama.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/attn_bench.py --batch 16 --seq 4096 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms split_dq16 split_dq16_dkv16 --rounds 3 > $O/ab_llama4k.log 2>&1 || exit $?
grep -h '^{' $O/ab_*.log
