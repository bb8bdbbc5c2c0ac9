# Produce the TunableOp (hipBLASLt/rocBLAS solution) table for a bench config: tune_gemms.sh [batch] [model] [seq]
set -e
B=${1:-64}; M=${2:-gpt2-small}; S=${3:-1024}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
# heartbeat: tuning a large shape can stay silent for minutes
(while true; do date >> gpurun_out/tune/heartbeat.log; sleep 50; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=40 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/${M}_b${B}_s${S}.csv \
timeout -k 10 900 python bench.py --batch $B --model $M --seq $S --steps 2 --warmup 1 --gemm-tuning off > gpurun_out/tune/tune_b$B.log 2>&1
cp gpurun_out/tune/${M}_b${B}_s${S}0.csv bpe_transformer/ops/tuning/${M}_b${B}_s${S}.csv
timeout -k 10 300 python bench.py --batch $B --model $M --seq $S --steps 20 --warmup 5 > gpurun_out/tune/bench_tuned_b$B.log 2>&1
