# round-end rehearsal: smoke, the whole GPU suite, the headline bench twice, a kernel-trace step profile and the
# step's hardware counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fc_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/fc_smoke.log; exit 1; }
tail -2 gpurun_out/fc_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fc_suite.log 2>&1 || { echo SUITEFAIL; tail -40 gpurun_out/fc_suite.log; exit 1; }
tail -1 gpurun_out/fc_suite.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/fc_bench_$i.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/fc_bench_$i.log; exit 1; }
  tail -1 gpurun_out/fc_bench_$i.log | cut -c1-260
done
bash tools/gpu/prof_step.sh r3final > /dev/null 2>&1 || { echo PROFFAIL; exit 1; }
head -24 gpurun_out/prof_r3final.md
bash tools/gpu/step_pmc.sh > gpurun_out/fc_pmc.log 2>&1 || { echo PMCFAIL; tail -20 gpurun_out/fc_pmc.log; exit 1; }
head -40 gpurun_out/step_pmc/summary.txt
