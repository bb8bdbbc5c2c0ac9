# one-call check: attention tests + A/B vs the pre-change library (variant "old") + stamps, then the whole GPU
# suite, smoke, the headline bench twice and a kernel-trace step profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "flash or sdpa" > gpurun_out/t_flash.log 2>&1 || { echo FLASHFAIL; tail -30 gpurun_out/t_flash.log; exit 1; }
tail -1 gpurun_out/t_flash.log
BPE_HIP_VARIANT=stamps timeout -k 10 120 python benchmarks/attn_stamps.py 2>&1 | grep -v amdgpu.ids
for v in "" old "" old; do
  echo "== variant=${v:-new}"
  BPE_HIP_VARIANT=$v timeout -k 10 120 python benchmarks/attn_bench.py --batch 128 --bwd-ab --iters 10 --rounds 5 --bwd-arms split fused 2>/dev/null
  BPE_HIP_VARIANT=$v timeout -k 10 120 python benchmarks/attn_bench.py --batch 128 --fwd-ab --fwd-versions 8 2 --iters 10 --rounds 5 2>/dev/null
  BPE_HIP_VARIANT=$v timeout -k 10 120 python benchmarks/attn_bench.py --batch 32 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --iters 10 --rounds 3 --bwd-arms split 2>/dev/null
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
BPE_PARITY_LOG=gpurun_out/parity timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r4_suite.log 2>&1 || { echo SUITEFAIL; tail -40 gpurun_out/r4_suite.log; exit 1; }
tail -1 gpurun_out/r4_suite.log
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/r4_bench$i.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/r4_bench$i.log; exit 1; }; tail -1 gpurun_out/r4_bench$i.log | cut -c1-200; done
bash tools/gpu/prof_step.sh r4a | head -30
