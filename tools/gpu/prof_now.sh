set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python benchmarks/lm_head_bench.py > gpurun_out/lmhead.log 2>&1
timeout -k 10 300 python -m pytest tests/test_model_gpu.py -x -q > gpurun_out/t_model.log 2>&1
BPE_VOCAB_PAD=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_pad0.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_now.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_now -o prof -- python bench.py --steps 5 --warmup 3 > gpurun_out/prof_now.log 2>&1
