# TunableOp tables for the Llama-1.1B 65536-token micro-batches (s2048 B32, s4096 B16), then tuned benches of
# both against the 16384-token defaults (B8 / B4), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/tune_gemms.sh 32 llama-1.1b 2048 || exit 1
echo "tuned s2048 b32"
bash tools/gpu/tune_gemms.sh 16 llama-1.1b 4096 || exit 1
echo "tuned s4096 b16"
cp gpurun_out/tune/llama-1.1b_b32_s20480.csv bpe_transformer/ops/tuning/llama-1.1b_b32_s2048.csv
cp gpurun_out/tune/llama-1.1b_b16_s40960.csv bpe_transformer/ops/tuning/llama-1.1b_b16_s4096.csv
run() { tag=$1; shift; timeout -k 10 400 python bench.py --model llama-1.1b --steps 8 --warmup 3 "$@" > gpurun_out/lbb_$tag.log 2>&1 || { tail -20 gpurun_out/lbb_$tag.log; exit 1; }; echo "$tag: $(tail -1 gpurun_out/lbb_$tag.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["gemm_tuning"], d["dw_gemm_routes"])')"; }
run s2048_b8 --seq 2048 --batch 8
run s2048_b32 --seq 2048 --batch 32
run s4096_b4 --seq 4096 --batch 4
run s4096_b16 --seq 4096 --batch 16
run s4096_b16_fp8 --seq 4096 --batch 16 --precision fp8
run s2048_b8_2 --seq 2048 --batch 8
run s2048_b32_2 --seq 2048 --batch 32
