# forward v9 (row sum on the VALU) vs v8 (row sum by MFMA): tests + op-level A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fwd_versions or fwd_v4 or flash_attention" > gpurun_out/fv_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/fv_tests.log; exit 1; }
tail -1 gpurun_out/fv_tests.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --fwd-ab --fwd-versions 7 8 9 --rounds 7 2>&1 | grep shape | tee gpurun_out/fv_ab.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 32 --seq 2048 --heads 32 --kv-heads 4 --fwd-ab --fwd-versions 7 8 9 --rounds 5 2>&1 | grep shape | tee -a gpurun_out/fv_ab.log
