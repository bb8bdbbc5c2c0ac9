# rocprofv3 hardware counters over one GPT-2 B128 training step (bench.py), three passes of kernel trace +
# counters only (never with sys/runtime traces), summarised per kernel by bpe_transformer.utils.pmc.
# usage (GPU box): bash tools/gpu/step_pmc.sh [bench args...]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$PWD/gpurun_out/step_pmc
rm -rf $OUT && mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --steps 1 --warmup 1 $*"
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o run \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -- python3 $B > $OUT/p1.log 2>&1
echo "pass 1 done"
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 -o run \
  --pmc FETCH_SIZE TCC_HIT_sum -- python3 $B > $OUT/p2.log 2>&1
echo "pass 2 done"
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p3 -o run \
  --pmc WRITE_SIZE TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -- python3 $B > $OUT/p3.log 2>&1
echo "pass 3 done"
python3 -m bpe_transformer.utils.pmc $OUT/p1 $OUT/p2 $OUT/p3 > $OUT/summary.txt
find $OUT -name "*.csv" -size +20M -delete
head -c 3000 $OUT/summary.txt
