# training-parity curves (fused engine vs eager PyTorch), the full GPU suite, the headline bench and a
# kernel-trace step profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BPE_PARITY_LOG=gpurun_out/parity timeout -k 10 300 python -u -m pytest tests/test_training_parity_gpu.py -x -v --timeout 280 --timeout-method thread > gpurun_out/t_parity.log 2>&1
rc=$?
if [ $rc -ne 0 ]; then
  echo "PARITYFAIL rc=$rc"; tail -30 gpurun_out/t_parity.log
  [ $rc -eq 1 ] || exit 1   # an assertion failure goes on; a timeout / crash ends the call
fi
timeout -k 10 900 python -u -m pytest tests -m gpu --deselect tests/test_training_parity_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo SUITEFAIL; tail -40 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_b128.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/bench_b128.log; exit 1; }
tail -1 gpurun_out/bench_b128.log
bash tools/gpu/prof_step.sh r3a
