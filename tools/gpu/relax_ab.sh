# spread-schedule phase-2 wait vmcnt(6) (default) vs vmcnt(4) (variant norelax): GEMM tests, op-level and e2e A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or swiglu or fp8 or rope or adamw" > gpurun_out/t_gemm.log 2>&1 || { echo GEMMFAIL; tail -30 gpurun_out/t_gemm.log; exit 1; }
tail -1 gpurun_out/t_gemm.log
timeout -k 10 120 python tools/gpu/dbg_persist.py 2>&1 | grep -v amdgpu.ids
for v in "" norelax "" norelax; do
  echo "== ${v:-relax}"
  BPE_HIP_VARIANT=$v timeout -k 10 300 python benchmarks/gemm_persist_ab.py --rounds 3 2>&1 | grep -v amdgpu.ids | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['op'][:28].ljust(28), d['persist_ms'])"
done
for v in "" norelax "" norelax; do
  BPE_HIP_VARIANT=$v timeout -k 10 300 python bench.py > gpurun_out/rx.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/rx.log; exit 1; }
  echo "${v:-relax} $(tail -1 gpurun_out/rx.log | cut -c1-140)"
done
bash tools/gpu/prof_step.sh r4d | head -30
