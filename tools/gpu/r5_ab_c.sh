#!/bin/bash
# round 5, call C: early closing barrier in the ping-pong GEMM (variant noeb = without) and prologue priority in the
# attention kernels (variant noprio = without): correctness, op-level, stamps, end to end.  Alternating, one box.
mkdir -p gpurun_out/abc
O=gpurun_out/abc
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm or flash or dq16" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for r in 1 2; do
  for V in default noeb; do
    E=""; [ $V != default ] && E="BPE_HIP_VARIANT=$V"
    env $E timeout -k 10 300 python -u benchmarks/gemm_pp_bench.py --model gpt2 --quick > $O/gemm_${V}_$r.log 2>&1 || exit $?
  done
  for V in default noprio; do
    E=""; [ $V != default ] && E="BPE_HIP_VARIANT=$V"
    env $E timeout -k 10 120 python -u benchmarks/attn_bench.py --batch 128 --iters 20 > $O/attn_${V}_$r.log 2>&1 || exit $?
    env $E timeout -k 10 120 python -u benchmarks/attn_bench.py --batch 32 --seq 2048 --heads 32 --kv-heads 4 --iters 10 > $O/attn_llama_${V}_$r.log 2>&1 || exit $?
  done
done
BPE_HIP_VARIANT=stamps timeout -k 10 120 python3 benchmarks/attn_stamps.py --dq-form 1 > $O/attn_stamps_f1_prio.log 2>&1 || exit $?
BPE_HIP_VARIANT=pstamps timeout -k 10 180 python3 benchmarks/gemm_phase_stamps.py > $O/gemm_phase_stamps_eb.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/e2e_default_$r.log 2>&1 || exit $?
  BPE_HIP_VARIANT=noeb timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/e2e_noeb_$r.log 2>&1 || exit $?
  BPE_HIP_VARIANT=noprio timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/e2e_noprio_$r.log 2>&1 || exit $?
done
grep -h '"metric"' $O/e2e_*.log | cut -c1-200
