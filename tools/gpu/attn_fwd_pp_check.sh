# ping-pong forward (v5): forward numerics, then the forward A/B (v2 / v4 / v5) at the GPT-2 B128 and Llama shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "flash" --timeout 120 --timeout-method thread > gpurun_out/t_fpp.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_fpp.log; exit 1; }
tail -2 gpurun_out/t_fpp.log
timeout -k 10 300 python benchmarks/attn_bench.py --batch 128 --fwd-ab --iters 10 > gpurun_out/abf.log 2>&1 &&
timeout -k 10 300 python benchmarks/attn_bench.py --batch 8 --seq 2048 --heads 32 --kv-heads 4 --fwd-ab --iters 10 >> gpurun_out/abf.log 2>&1
rc=$?
grep fwd_version gpurun_out/abf.log
exit $rc
