# rocprofv3 kernel stats + counter passes over the attention microbenchmark (split backward), GPT-2 B128 shape.
# usage (GPU box): bash tools/gpu/attn_split_pmc.sh [extra attn_bench args]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$PWD/gpurun_out/attn_pmc
rm -rf $OUT && mkdir -p $OUT
export TMPDIR=/tmp
ARGS="benchmarks/attn_bench.py --batch 128 --iters 3 $*"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/st -o run -- python3 $ARGS > $OUT/st.log 2>&1
echo "stats done"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o run \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -- python3 $ARGS > $OUT/p1.log 2>&1
echo "pass 1 done"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 -o run \
  --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -- python3 $ARGS > $OUT/p2.log 2>&1
echo "pass 2 done"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p3 -o run \
  --pmc FETCH_SIZE TCC_HIT_sum -- python3 $ARGS > $OUT/p3.log 2>&1
echo "pass 3 done"
python3 -m bpe_transformer.utils.pmc $OUT/p1 $OUT/p2 $OUT/p3 --match fa_ > $OUT/summary.txt
find $OUT -name "*.csv" -size +20M -delete
cat $OUT/summary.txt
find $OUT/st -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -20
timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --bwd-ab --iters 10 > $OUT/ab.log 2>&1
cat $OUT/ab.log
