#!/bin/bash
# round-5 end: re-tune the Llama-1.1B s2048 B32 / s4096 B16 TunableOp tables on the current tree, A/B against the shipped
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/retune_llama
mkdir -p $O
(while true; do date >> $O/heartbeat.log; sleep 50; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for cfg in "b32_s2048:2048" "b16_s4096:4096"; do
  tag=${cfg%%:*}; S=${cfg#*:}
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=40 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
  PYTORCH_TUNABLEOP_FILENAME=$O/llama-1.1b_$tag.csv \
  timeout -k 10 900 python bench.py --model llama-1.1b --seq $S --steps 2 --warmup 1 --gemm-tuning off > $O/tune_$tag.log 2>&1 || { echo TUNEFAIL; tail -20 $O/tune_$tag.log; exit 1; }
done
ls $O
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --model llama-1.1b "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; return 1; }
  tail -n 1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"], d.get("gemm_tuning"))' $tag | tee -a $O/summary.log
}
for r in 1 2; do
  run new_s2048_$r --seq 2048 --gemm-tuning $(ls $O/llama-1.1b_b32_s2048*.csv | head -1) || exit 1
  run old_s2048_$r --seq 2048 || exit 1
done
run new_s4096_1 --seq 4096 --gemm-tuning $(ls $O/llama-1.1b_b16_s4096*.csv | head -1) || exit 1
run old_s4096_1 --seq 4096 || exit 1
