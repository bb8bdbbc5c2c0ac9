#!/bin/bash
# round-5 end rehearsal: smoke, the whole GPU suite, the headline bench twice (the driver's own sequence)
set -o pipefail
mkdir -p gpurun_out/final
O=gpurun_out/final
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 1; }
tail -n 2 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { echo SUITEFAIL; tail -40 $O/suite.log; exit 1; }
tail -n 1 $O/suite.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || { echo BENCHFAIL; tail -20 $O/bench_$i.log; exit 1; }
  tail -n 1 $O/bench_$i.log | cut -c1-300
done
