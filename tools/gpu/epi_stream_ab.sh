# SwiGLU-backward epilogue streaming its g/u loads (in-tree) vs the drained version (variant "pre"): numerics,
# op-level A/B, end to end A/B (alternating)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "swiglu or gemm_pp" --timeout 120 --timeout-method thread > gpurun_out/t_epi.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_epi.log; exit 1; }
tail -1 gpurun_out/t_epi.log
for v in pre new pre new; do
  if [ $v = pre ]; then export BPE_HIP_VARIANT=pre; else unset BPE_HIP_VARIANT; fi
  timeout -k 10 200 python benchmarks/swiglu_bench.py > gpurun_out/epi_sw_$v.log 2>&1 || { tail -20 gpurun_out/epi_sw_$v.log; exit 1; }
  echo "$v: $(grep -E 'fused' gpurun_out/epi_sw_$v.log | python3 -c 'import sys,json; print([(json.loads(l)["op"], json.loads(l)["ms"]) for l in sys.stdin])')"
done
for v in pre new pre new; do
  if [ $v = pre ]; then export BPE_HIP_VARIANT=pre; else unset BPE_HIP_VARIANT; fi
  timeout -k 10 300 python bench.py > gpurun_out/epi_bench_$v.log 2>&1 || { tail -20 gpurun_out/epi_bench_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/epi_bench_$v.log | cut -c1-200)"
done
