#!/bin/bash
# round 5: the non-temporal hint on the streaming kernels (BPE_STREAM_NT: CE, RMSNorm backward, the SwiGLU-backward
# GEMM epilogue) -- default (on) vs variant nont (off), op-level fused GEMMs and end to end, alternating
mkdir -p gpurun_out/snt
O=gpurun_out/snt
for r in 1 2; do
  for V in default nont; do
    E=""; [ $V != default ] && E="BPE_HIP_VARIANT=$V"
    env $E timeout -k 10 200 python -u benchmarks/gemm_fused_ab.py >> $O/fused_$V.log 2>&1 || exit $?
  done
done
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/e2e_default_$r.log 2>&1 || exit $?
  BPE_HIP_VARIANT=nont timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/e2e_nont_$r.log 2>&1 || exit $?
done
grep -h '^{' $O/fused_*.log; grep -h '"metric"' $O/e2e_*.log | cut -c1-160
