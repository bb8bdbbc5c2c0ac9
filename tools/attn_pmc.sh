# rocprofv3 counter passes over the attention microbenchmark (one pass per counter set, kernel trace only)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="benchmarks/attn_bench.py --batch 64 --iters 2 ${ATTN_ARGS:-}"
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o run \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -- python3 $ARGS
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 -o run \
  --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -- python3 $ARGS
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/p3 -o run \
  --pmc SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INST_LEVEL_VMEM -- python3 $ARGS
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/p4 -o run \
  --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum -- python3 $ARGS
python3 -m bpe_transformer.utils.pmc $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 --match fa_ > $OUT/summary.txt
cat $OUT/summary.txt
