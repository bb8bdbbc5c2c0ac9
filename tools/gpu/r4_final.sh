# round-4 check at HEAD: smoke, full GPU suite (parity curves), headline bench twice, step profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
BPE_PARITY_LOG=gpurun_out/parity timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r4_suite.log 2>&1 || { echo SUITEFAIL; tail -40 gpurun_out/r4_suite.log; exit 1; }
tail -1 gpurun_out/r4_suite.log
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/r4_bench$i.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/r4_bench$i.log; exit 1; }; tail -1 gpurun_out/r4_bench$i.log | cut -c1-200; done
bash tools/gpu/prof_step.sh r4c | head -12
