#!/bin/bash
# round 5: the A prefetch (PREA) on the fused ping-pong GEMMs and the fp8 hand kernel, alternating with variant noprea
mkdir -p gpurun_out/prea
O=gpurun_out/prea
for r in 1 2 3; do
  for V in default noprea; do
    E=""; [ $V != default ] && E="BPE_HIP_VARIANT=$V"
    env $E timeout -k 10 200 python -u benchmarks/gemm_fused_ab.py >> $O/gpt2_$V.log 2>&1 || exit $?
    env $E timeout -k 10 200 python -u benchmarks/gemm_fused_ab.py --tokens 65536 --d 2048 --ff 5632 --seq 4096 --reps 10 >> $O/llama_$V.log 2>&1 || exit $?
  done
done
grep -h '^{' $O/*.log
