#!/bin/bash
# round 5: TunableOp table for the fp8 Llama config (hipBLASLt's _scaled_mm solutions), merged into the s4096 B16 table,
# then same-box A/B of the fp8 config with the old and the merged table (alternating)
set -e
mkdir -p gpurun_out/tune
(while true; do date >> gpurun_out/tune/heartbeat.log; sleep 50; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
OLD=bpe_transformer/ops/tuning/llama-1.1b_b16_s4096.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=40 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/fp8_s4096_b16.csv \
timeout -k 10 900 python bench.py --model llama-1.1b --seq 4096 --precision fp8 --steps 2 --warmup 1 --gemm-tuning off > gpurun_out/tune/tune_fp8.log 2>&1
NEW=$(ls gpurun_out/tune/fp8_s4096_b16*.csv | head -1)
python - "$OLD" "$NEW" gpurun_out/tune/merged_s4096_b16.csv <<'PY'
import sys
old, new, out = sys.argv[1:]
rows = {}
order = []
for path in (old, new):
    for line in open(path):
        parts = line.rstrip("\n").split(",")
        if len(parts) < 2:
            continue
        key = (parts[0], parts[1])
        if key not in rows:
            order.append(key)
        if parts[0] == "Validator" and key in rows:
            continue
        if path == new and parts[0] != "Validator" and not parts[0].startswith("ScaledGemm") and key in rows:
            continue  # keep the bf16 run's own solutions for the bf16 shapes
        rows[key] = line.rstrip("\n")
open(out, "w").write("\n".join(rows[k] for k in order) + "\n")
print("merged", len(rows), "rows;", sum(1 for k in rows if k[0].startswith("ScaledGemm")), "scaled-gemm rows")
PY
for i in 1 2; do
  timeout -k 10 300 python bench.py --model llama-1.1b --seq 4096 --precision fp8 --steps 10 --warmup 3 > gpurun_out/tune/ab_old_$i.log 2>&1
  timeout -k 10 300 python bench.py --model llama-1.1b --seq 4096 --precision fp8 --steps 10 --warmup 3 --gemm-tuning gpurun_out/tune/merged_s4096_b16.csv > gpurun_out/tune/ab_new_$i.log 2>&1
done
