#!/bin/bash
# round-5 end: re-tune the GPT-2 B 128 TunableOp table on the current tree, then A/B it against the shipped table
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/retune
mkdir -p $O
(while true; do date >> $O/heartbeat.log; sleep 50; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=40 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
PYTORCH_TUNABLEOP_FILENAME=$O/gpt2-small_b128_s1024.csv \
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --gemm-tuning off > $O/tune.log 2>&1 || { echo TUNEFAIL; tail -20 $O/tune.log; exit 1; }
ls $O
NEW=$(ls $O/gpt2-small_b128_s1024*.csv | head -1)
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; return 1; }
  tail -n 1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"], d.get("gemm_tuning"))' $tag | tee -a $O/summary.log
}
for r in 1 2; do
  run new_$r --gemm-tuning $NEW || exit 1
  run old_$r || exit 1
done
