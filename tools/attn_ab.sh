set -e
for g in 0 16 64 256; do
  for v3 in 1 0; do
    echo "group=$g v3=$v3 $(BPE_FA_GROUP=$g BPE_FA_FWD_V3=$v3 python -u benchmarks/attn_bench.py --batch 128 --no-rope)"
  done
done
echo "rope block g64 $(python -u benchmarks/attn_bench.py --batch 128)"
echo "rope fused g64 $(python -u benchmarks/attn_bench.py --batch 128 --mode fused)"
