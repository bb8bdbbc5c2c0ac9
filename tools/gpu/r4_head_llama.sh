# LM-head GEMMs on the persistent kernel vs hipBLASLt; Llama SwiGLU forward fusion cap re-A/B (persistent kernel);
# full GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/gemm_persist_ab.py --head --rounds 3 2>&1 | grep -v amdgpu.ids
B="--model llama-1.1b --seq 2048 --steps 10 --warmup 3"
for i in 1 2; do
  timeout -k 10 400 python bench.py $B > gpurun_out/ll.log 2>&1 || { echo LLFAIL; tail -20 gpurun_out/ll.log; exit 1; }
  echo "llama cap1024  $(tail -1 gpurun_out/ll.log | cut -c1-150)"
  timeout -k 10 400 python benchmarks/bench_ab.py --set bpe_transformer.models.fused_block._FUSE_SWIGLU_FWD_MAX_D=4096 -- $B > gpurun_out/ll.log 2>&1 || { echo LLFAIL; tail -20 gpurun_out/ll.log; exit 1; }
  echo "llama cap4096  $(tail -1 gpurun_out/ll.log | cut -c1-150)"
done
BPE_PARITY_LOG=gpurun_out/parity timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r4_suite.log 2>&1 || { echo SUITEFAIL; tail -40 gpurun_out/r4_suite.log; exit 1; }
tail -1 gpurun_out/r4_suite.log
