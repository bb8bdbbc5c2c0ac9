#!/bin/bash
# round 5: prologue operands kept before the barrier (fa_common.h keep) -- default vs variant prev (the previous
# commit's kernels): attention tests, op-level fwd / bwd, stamps, end to end.  Alternating, one box.
mkdir -p gpurun_out/keep
O=gpurun_out/keep
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "flash" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for r in 1 2 3; do
  for V in default prev; do
    E=""; [ $V != default ] && E="BPE_HIP_VARIANT=$V"
    env $E timeout -k 10 120 python -u benchmarks/attn_bench.py --batch 128 --iters 20 >> $O/attn_gpt2_$V.log 2>&1 || exit $?
    env $E timeout -k 10 120 python -u benchmarks/attn_bench.py --batch 32 --seq 2048 --heads 32 --kv-heads 4 --iters 10 >> $O/attn_llama_$V.log 2>&1 || exit $?
  done
done
BPE_HIP_VARIANT=stamps timeout -k 10 120 python3 benchmarks/attn_stamps.py --dq-form 1 > $O/stamps_f1.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/e2e_default_$r.log 2>&1 || exit $?
  BPE_HIP_VARIANT=prev timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/e2e_prev_$r.log 2>&1 || exit $?
done
grep -h '^{' $O/attn_*.log | cut -c1-200; head -3 $O/stamps_f1.log; grep -h '"metric"' $O/e2e_*.log | cut -c1-160
