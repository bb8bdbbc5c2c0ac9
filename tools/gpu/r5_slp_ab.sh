#!/bin/bash
# round 5: packed-f32 VALU off in the MFMA kernels (per-file -fno-slp-vectorize, default build) vs on (variant slp);
# the 16-queries-per-wave dQ kernel end to end.  Alternating, one box.
mkdir -p gpurun_out/slp
O=gpurun_out/slp
for r in 1 2; do
  for V in default slp; do
    E=""; [ $V = slp ] && E="BPE_HIP_VARIANT=slp"
    env $E timeout -k 10 120 python -u benchmarks/attn_bench.py --batch 128 --iters 20 > $O/attn_${V}_$r.log 2>&1 || exit $?
    env $E timeout -k 10 300 python -u benchmarks/gemm_pp_bench.py --model gpt2 --quick > $O/gemm_${V}_$r.log 2>&1 || exit $?
  done
done
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/e2e_default_$r.log 2>&1 || exit $?
  BPE_HIP_VARIANT=slp timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/e2e_slp_$r.log 2>&1 || exit $?
  timeout -k 10 400 python -u benchmarks/bench_ab.py --op fa_dq_config=1 -- --steps 20 --warmup 5 > $O/e2e_dq16_$r.log 2>&1 || exit $?
done
grep -h "ms" $O/attn_*.log; grep -h '"metric"' $O/e2e_*.log
