#!/bin/bash
# round 5, call B: end to end (bench.py GPT-2 B 128, 20 steps) -- HEAD, no A prefetch, packed f32 VALU, dq16
mkdir -p gpurun_out/ab
O=gpurun_out/ab
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/e2e_default_$r.log 2>&1 || exit $?
  BPE_HIP_VARIANT=noprea timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/e2e_noprea_$r.log 2>&1 || exit $?
  BPE_HIP_VARIANT=slp timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/e2e_slp_$r.log 2>&1 || exit $?
  timeout -k 10 300 python -u benchmarks/bench_ab.py --op fa_dq_config=1 -- --steps 20 --warmup 5 > $O/e2e_dq16_$r.log 2>&1 || exit $?
done
grep -h '"metric"' $O/e2e_*.log
