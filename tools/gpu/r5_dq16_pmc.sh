#!/bin/bash
# round 5: counters of the 32- and 16-queries-per-wave dQ kernels (GPT-2 B 128), the fixed LDS-DMA issue microbench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/dq16_pmc
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 120 ./benchmarks/dma_issue_bench.bin > gpurun_out/dma_issue_bench_fixed.log 2>&1 || exit $?
for F in 0 1; do
  ARGS="benchmarks/attn_bench.py --batch 128 --iters 3 --dq-form $F"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/f$F/p1 -o run \
    --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -- python3 $ARGS > $OUT/f$F.p1.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/f$F/p2 -o run \
    --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -- python3 $ARGS > $OUT/f$F.p2.log 2>&1 || exit $?
  python3 -m bpe_transformer.utils.pmc $OUT/f$F/p1 $OUT/f$F/p2 --match fa_bwd > $OUT/summary_f$F.txt || exit $?
done
find $OUT -name "*.csv" -size +20M -delete
cat $OUT/summary_f0.txt $OUT/summary_f1.txt
for F in 0 1; do
  BPE_HIP_VARIANT=stamps timeout -k 10 120 python3 benchmarks/attn_stamps.py --dq-form $F > gpurun_out/attn_stamps_f$F.log 2>&1 || exit $?
  BPE_HIP_VARIANT=stamps timeout -k 10 120 python3 benchmarks/attn_stamps.py --dq-form $F --batch 32 --seq 2048 --heads 32 --kv-heads 4 > gpurun_out/attn_stamps_llama_f$F.log 2>&1 || exit $?
done
cat gpurun_out/attn_stamps_f*.log
BPE_HIP_VARIANT=pstamps timeout -k 10 180 python3 benchmarks/gemm_phase_stamps.py > gpurun_out/gemm_phase_stamps.log 2>&1 || exit $?
cat gpurun_out/gemm_phase_stamps.log
