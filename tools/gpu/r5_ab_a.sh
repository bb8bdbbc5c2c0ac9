#!/bin/bash
# round 5, call A: GEMM / attention correctness on the A-prefetch build, op-level A/B of the A prefetch (variant
# noprea), of packed f32 VALU (variant slp), phase stamps of the new schedule
mkdir -p gpurun_out/ab
O=gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm or flash_bwd_split or dq16" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
tail -n 2 $O/tests.log
for r in 1 2; do
  for V in default noprea slp; do
    E=""; [ $V != default ] && E="BPE_HIP_VARIANT=$V"
    env $E timeout -k 10 300 python -u benchmarks/gemm_pp_bench.py --model gpt2 --quick > $O/gemm_${V}_$r.log 2>&1 || exit $?
  done
  for V in default slp; do
    E=""; [ $V != default ] && E="BPE_HIP_VARIANT=$V"
    env $E timeout -k 10 120 python -u benchmarks/attn_bench.py --batch 128 --iters 20 > $O/attn_${V}_$r.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python -u benchmarks/attn_bench.py --batch 128 --bwd-ab --bwd-arms split split_dq16 split_dq16_nw4 --rounds 5 > $O/dq_forms_gpt2.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/attn_bench.py --batch 32 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms split split_dq16 split_dq16_nw4 --rounds 5 > $O/dq_forms_llama.log 2>&1 || exit $?
BPE_HIP_VARIANT=stamps timeout -k 10 120 python3 benchmarks/attn_stamps.py --dq-form 2 > $O/attn_stamps_f2.log 2>&1 || exit $?
BPE_HIP_VARIANT=pstamps timeout -k 10 180 python3 benchmarks/gemm_phase_stamps.py > $O/gemm_phase_stamps_prea.log 2>&1 || exit $?
grep -h "ms" $O/attn_*.log $O/dq_forms_*.log
