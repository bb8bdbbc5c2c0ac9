# persistent gemm_pp: GEMM tests, stamps of both forms, op-level A/B (GPT-2 and Llama shapes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/gpu/dbg_persist.py 2>&1 | grep -v amdgpu.ids && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or swiglu or fp8" > gpurun_out/t_gemm.log 2>&1 || { echo GEMMFAIL; tail -30 gpurun_out/t_gemm.log; exit 1; }
tail -1 gpurun_out/t_gemm.log
BPE_HIP_VARIANT=stamps timeout -k 10 200 python benchmarks/gemm_stamps.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python benchmarks/gemm_persist_ab.py --model gpt2 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python benchmarks/gemm_persist_ab.py --model llama --tokens 65536 --rounds 3 2>&1 | grep -v amdgpu.ids
