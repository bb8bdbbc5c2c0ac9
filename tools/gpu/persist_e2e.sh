# persistent gemm_pp end to end: GEMM A/B incl. the input-gradient shapes, then the headline bench alternating
# the default library (persistent) with the one-tile variant build (BPE_HIP_VARIANT=tile), twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/gemm_persist_ab.py --model gpt2 --rounds 3 2>&1 | grep -v amdgpu.ids
for v in "" tile "" tile; do
  BPE_HIP_VARIANT=$v timeout -k 10 300 python bench.py > gpurun_out/pe_bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/pe_bench.log; exit 1; }
  echo "variant=${v:-persist} $(tail -1 gpurun_out/pe_bench.log | cut -c1-150)"
done
