# forward v5 numerics + A/B, then the full GPU suite (training parity curves logged), the headline bench and a
# kernel-trace step profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu/attn_fwd_pp_check.sh || exit 1
BPE_PARITY_LOG=gpurun_out/parity timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo SUITEFAIL; tail -40 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_b128.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/bench_b128.log; exit 1; }
tail -1 gpurun_out/bench_b128.log
bash tools/gpu/prof_step.sh r3a
