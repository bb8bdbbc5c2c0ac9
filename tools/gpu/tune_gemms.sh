# Produce the TunableOp (hipBLASLt/rocBLAS solution) table for the headline bench config.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=40 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/gpt2-small_b64_s1024.csv \
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --gemm-tuning off > gpurun_out/tune/tune.log 2>&1
cp gpurun_out/tune/gpt2-small_b64_s10240.csv bpe_transformer/ops/tuning/gpt2-small_b64_s1024.csv
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/tune/bench_tuned.log 2>&1
