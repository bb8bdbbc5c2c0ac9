#!/bin/bash
# round 5: non-temporal loads / stores in the 128 x 128 fp8 casts (variant nont = without): tests, op-level, fp8 step
mkdir -p gpurun_out/fp8nt
O=gpurun_out/fp8nt
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "cast or swiglu" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for r in 1 2; do
  for V in default nont; do
    E=""; [ $V != default ] && E="BPE_HIP_VARIANT=$V"
    env $E timeout -k 10 200 python -u benchmarks/cast_bench.py > $O/cast_${V}_$r.log 2>&1 || exit $?
  done
done
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --model llama-1.1b --seq 4096 --precision fp8 --steps 10 --warmup 3 > $O/e2e_default_$r.log 2>&1 || exit $?
  BPE_HIP_VARIANT=nont timeout -k 10 400 python -u bench.py --model llama-1.1b --seq 4096 --precision fp8 --steps 10 --warmup 3 > $O/e2e_nont_$r.log 2>&1 || exit $?
done
grep -h swiglu $O/cast_*.log; grep -h '"metric"' $O/e2e_*.log | cut -c1-160
