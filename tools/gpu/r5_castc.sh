#!/bin/bash
# coalesced-load 128 x 128 fp8 casts (fp8_cast_config 1) vs row pairs (0): bitwise test, then the cast bench
set -o pipefail
O=gpurun_out/castc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fp8_cast_forms or cast_fp8 or swiglu_cast" > $O/test.log 2>&1 || { echo TESTFAIL; tail -30 $O/test.log; exit 1; }
tail -n 1 $O/test.log
timeout -k 10 300 python benchmarks/cast_bench.py --forms 0,1,2 > $O/bench.log 2>&1 || { echo BENCHFAIL; tail -20 $O/bench.log; exit 1; }
cat $O/bench.log | grep -v amdgpu.ids
for r in 1 2; do
  for F in 0 2; do
    timeout -k 10 400 python -u benchmarks/bench_ab.py --op fp8_cast_config=$F -- --model llama-1.1b --seq 4096 --precision fp8 --steps 10 --warmup 3 > $O/e2e_f${F}_$r.log 2>&1 || { echo E2EFAIL; tail -20 $O/e2e_f${F}_$r.log; exit 1; }
    echo "f$F $(grep -h '"metric"' $O/e2e_f${F}_$r.log | cut -c1-200)"
  done
done
