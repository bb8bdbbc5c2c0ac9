#!/bin/bash
# coalesced 128 x 128 fp8 casts as the only form: fp8 tests, cast bench, fp8 Llama step
set -o pipefail
O=gpurun_out/castd
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fp8 or cast" > $O/test.log 2>&1 || { echo TESTFAIL; tail -30 $O/test.log; exit 1; }
tail -n 1 $O/test.log
timeout -k 10 300 python benchmarks/cast_bench.py > $O/bench.log 2>&1 || { echo BENCHFAIL; tail -20 $O/bench.log; exit 1; }
grep -v amdgpu.ids $O/bench.log
timeout -k 10 400 python -u bench.py --model llama-1.1b --seq 4096 --precision fp8 --steps 10 --warmup 3 > $O/e2e.log 2>&1 || { echo E2EFAIL; tail -20 $O/e2e.log; exit 1; }
grep -h '"metric"' $O/e2e.log | cut -c1-200
