# packed masked paths in dK/dV and dQ (HEAD tree) vs the previous commit (variant prevm2): tests + op-level A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash_bwd or flash_attention" > gpurun_out/m2_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/m2_tests.log; exit 1; }
tail -1 gpurun_out/m2_tests.log
for v in "" prevm2 "" prevm2; do
  BPE_HIP_VARIANT=$v timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --bwd-ab --bwd-arms 48,44 --rounds 5 2>&1 | grep shape | sed "s/^/[${v:-head}] /" | tee -a gpurun_out/m2_ab.log
  BPE_HIP_VARIANT=$v timeout -k 10 300 python benchmarks/attn_bench.py --batch 32 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms 48,44 --rounds 3 2>&1 | grep shape | sed "s/^/[${v:-head}] /" | tee -a gpurun_out/m2_ab.log
done
