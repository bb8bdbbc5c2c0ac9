# single-compare causal masks (HEAD tree) vs the previous commit's kernels (variant prevmask): tests + op-level A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > gpurun_out/mk_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/mk_tests.log; exit 1; }
tail -1 gpurun_out/mk_tests.log
for v in "" prevmask "" prevmask; do
  BPE_HIP_VARIANT=$v timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --fwd-ab --fwd-versions 7 8 --bwd-ab --bwd-arms 44,44 --rounds 5 2>&1 | grep shape | sed "s/^/[${v:-head}] /" | tee -a gpurun_out/mk_ab.log
done
