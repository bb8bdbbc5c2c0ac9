# session start: smoke, the whole GPU suite, the headline bench once
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/sc_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/sc_smoke.log; exit 1; }
tail -2 gpurun_out/sc_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/sc_suite.log 2>&1 || { echo SUITEFAIL; tail -40 gpurun_out/sc_suite.log; exit 1; }
tail -1 gpurun_out/sc_suite.log
timeout -k 10 300 python bench.py > gpurun_out/sc_bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/sc_bench.log; exit 1; }
tail -2 gpurun_out/sc_bench.log | cut -c1-400
