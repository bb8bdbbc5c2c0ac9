# forward versions: tests, then op-level A/B (GPT-2 B 128 and Llama GQA shapes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fwd_versions or fwd_v4 or flash_attention" > gpurun_out/af_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/af_tests.log; exit 1; }
tail -1 gpurun_out/af_tests.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --fwd-ab --fwd-versions 4 6 7 --rounds 7 > gpurun_out/af_fwd.log 2>&1 || { echo FWDFAIL; tail gpurun_out/af_fwd.log; exit 1; }
grep -v amdgpu.ids gpurun_out/af_fwd.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 8 --seq 2048 --heads 32 --kv-heads 4 --fwd-ab --fwd-versions 4 6 7 --rounds 7 > gpurun_out/af_fwd_llama.log 2>&1 || { echo FWDFAIL2; tail gpurun_out/af_fwd_llama.log; exit 1; }
grep -v amdgpu.ids gpurun_out/af_fwd_llama.log
