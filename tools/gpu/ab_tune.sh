set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_tuned.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --gemm-tuning off > gpurun_out/ab_untuned.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_tuned2.log 2>&1
