#!/bin/bash
# round-5 end: GPT-2 step profile at HEAD, then the driver's sequence (smoke, GPU suite, bench x2)
set -o pipefail
bash tools/gpu/prof_step.sh r5end > /dev/null 2>&1 || { echo PROFFAIL; tail -20 gpurun_out/prof_r5end.log; exit 1; }
head -20 gpurun_out/prof_r5end.md
bash tools/gpu/r5_final.sh
