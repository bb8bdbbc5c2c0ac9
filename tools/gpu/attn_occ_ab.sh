# LDS-DMA-staged split backward (42 / 43) and the 3-waves-per-SIMD forward (v6): correctness, then op-level A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash_bwd_split or fwd_versions or flash_attention" > gpurun_out/ao_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/ao_tests.log; exit 1; }
tail -1 gpurun_out/ao_tests.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --fwd-ab --fwd-versions 4 6 --rounds 5 > gpurun_out/ao_fwd.log 2>&1 || { echo FWDFAIL; tail gpurun_out/ao_fwd.log; exit 1; }
cat gpurun_out/ao_fwd.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --bwd-ab --bwd-arms split4x4 42,42 42,4 4,42 43,43 --rounds 5 > gpurun_out/ao_bwd.log 2>&1 || { echo BWDFAIL; tail gpurun_out/ao_bwd.log; exit 1; }
cat gpurun_out/ao_bwd.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 8 --seq 2048 --heads 32 --kv-heads 4 --bwd-ab --bwd-arms split4x4 42,42 43,43 --rounds 5 > gpurun_out/ao_bwd_llama.log 2>&1 || { echo BWDFAIL2; tail gpurun_out/ao_bwd_llama.log; exit 1; }
cat gpurun_out/ao_bwd_llama.log
