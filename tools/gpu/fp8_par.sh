set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
BPE_PARITY_LOG=gpurun_out/parity timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/test_training_parity_gpu.py -k fp8 > gpurun_out/t_fp8par.log 2>&1 || { echo PARFAIL; tail -30 gpurun_out/t_fp8par.log; exit 1; }
tail -1 gpurun_out/t_fp8par.log
