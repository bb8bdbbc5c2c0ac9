# same-box A/B of the flat gradient buffer dtype (bf16 default vs fp32) at the headline config, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
for gd in bf16 fp32 bf16 fp32; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --grad-dtype $gd > gpurun_out/bench_gd_$gd.log 2>&1 || { tail -20 gpurun_out/bench_gd_$gd.log; exit 1; }
  echo "$gd: $(tail -1 gpurun_out/bench_gd_$gd.log)"
done
