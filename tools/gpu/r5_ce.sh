#!/bin/bash
# VALU-lean softmax-CE register kernel (default) vs the previous form (variant cenf): tests, op-level, e2e
set -o pipefail
O=gpurun_out/ce
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_training_parity_gpu.py -x -q --timeout 200 --timeout-method thread -k "cross_entropy or lm_head or ce_ or parity_gpt2 or loss" > $O/test.log 2>&1 || { echo TESTFAIL; tail -30 $O/test.log; exit 1; }
tail -n 1 $O/test.log
for r in 1 2 3; do
  for V in default cenf; do
    E=""; [ $V != default ] && E="BPE_HIP_VARIANT=$V"
    env $E timeout -k 10 200 python -u benchmarks/ce_bench.py --rows 131072 > $O/op_${V}_$r.log 2>&1 || { echo OPFAIL; tail -20 $O/op_${V}_$r.log; exit 1; }
    echo "$V $(grep -h TB_s $O/op_${V}_$r.log)"
  done
done
for r in 1 2; do
  for V in default cenf; do
    E=""; [ $V != default ] && E="BPE_HIP_VARIANT=$V"
    env $E timeout -k 10 300 python -u bench.py > $O/e2e_${V}_$r.log 2>&1 || { echo E2EFAIL; tail -20 $O/e2e_${V}_$r.log; exit 1; }
    echo "$V $(tail -n 1 $O/e2e_${V}_$r.log | cut -c1-190)"
  done
done
