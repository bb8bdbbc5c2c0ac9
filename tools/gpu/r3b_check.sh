# attention defaults (bwd 42,42 / fwd v7): full GPU suite, end-to-end A/B vs the previous defaults, step profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3b_suite.log 2>&1 || { echo SUITEFAIL; tail -40 gpurun_out/r3b_suite.log; exit 1; }
tail -1 gpurun_out/r3b_suite.log
bash tools/gpu/ab_env.sh "BPE_FA_SPLIT_NW=4,4 BPE_FA_FWD=4" "BPE_GPP_PRIO=1" "BPE_FA_SPLIT_NW=4,4 BPE_FA_FWD=4" "BPE_GPP_PRIO=1" > gpurun_out/ab_e2e_attn_defaults.log 2>&1 || { echo ABFAIL; cat gpurun_out/ab_e2e_attn_defaults.log; exit 1; }
cat gpurun_out/ab_e2e_attn_defaults.log
bash tools/gpu/prof_step.sh r3b > /dev/null 2>&1 || { echo PROFFAIL; tail gpurun_out/prof_r3b.log; exit 1; }
head -36 gpurun_out/prof_r3b.md
