# GQA dK / dV head sweep: tests, op-level A/B vs partials + reduce (Llama shape), Llama bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > gpurun_out/gq_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/gq_tests.log; exit 1; }
tail -1 gpurun_out/gq_tests.log
for loop in 1 0 1 0; do
  BPE_FA_GQA_LOOP=$loop timeout -k 10 300 python benchmarks/attn_bench.py --batch 32 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms 44,44 --rounds 5 2>&1 | grep shape | sed "s/^/loop=$loop /" | tee -a gpurun_out/gq_ab.log
done
bash tools/gpu/ab_env_args.sh "--model llama-1.1b --seq 2048 --steps 10 --warmup 3" "BPE_FA_GQA_LOOP=1" "BPE_FA_GQA_LOOP=0" "BPE_FA_GQA_LOOP=1" "BPE_FA_GQA_LOOP=0" 2>&1 | tee gpurun_out/gq_e2e.log
