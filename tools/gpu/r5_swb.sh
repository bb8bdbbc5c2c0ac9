#!/bin/bash
# early pass-1 g / u loads in the persistent SwiGLU-backward epilogue (default) vs the two-pass epilogue (variant swb0): tests, op-level, e2e
set -o pipefail
O=gpurun_out/swb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "swiglu or persist" > $O/test.log 2>&1 || { echo TESTFAIL; tail -30 $O/test.log; exit 1; }
tail -n 1 $O/test.log
for r in 1 2 3; do
  for V in default swb0; do
    E=""; [ $V != default ] && E="BPE_HIP_VARIANT=$V"
    env $E timeout -k 10 200 python -u benchmarks/gemm_fused_ab.py > $O/op_${V}_$r.log 2>&1 || { echo OPFAIL; tail -20 $O/op_${V}_$r.log; exit 1; }
    grep -h swiglu_fwd_us $O/op_${V}_$r.log
  done
done
for r in 1 2; do
  for V in default swb0; do
    E=""; [ $V != default ] && E="BPE_HIP_VARIANT=$V"
    env $E timeout -k 10 300 python -u bench.py > $O/e2e_${V}_$r.log 2>&1 || { echo E2EFAIL; tail -20 $O/e2e_${V}_$r.log; exit 1; }
    echo "$V $(tail -n 1 $O/e2e_${V}_$r.log | cut -c1-190)"
  done
done
