#!/bin/bash
# round 5: 32-row vs 16-row dQ kernel across sequence lengths (op-level, same process, interleaved)
mkdir -p gpurun_out/dqs
O=gpurun_out/dqs
timeout -k 10 200 python -u benchmarks/attn_bench.py --batch 16 --seq 4096 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms split split_dq16 --rounds 5 > $O/s4096.log 2>&1 || exit $?
timeout -k 10 200 python -u benchmarks/attn_bench.py --batch 4 --seq 8192 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms split split_dq16 --rounds 3 > $O/s8192.log 2>&1 || exit $?
timeout -k 10 200 python -u benchmarks/attn_bench.py --batch 32 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms split split_dq16 --rounds 5 > $O/s2048.log 2>&1 || exit $?
timeout -k 10 200 python -u benchmarks/attn_bench.py --batch 128 --bwd-ab --bwd-arms split split_dq16 --rounds 5 > $O/s1024.log 2>&1 || exit $?
grep -h '^{' $O/*.log
