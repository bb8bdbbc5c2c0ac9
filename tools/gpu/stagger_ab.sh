# fused SwiGLU GEMMs: first-wave stagger A/B (op level, GPT-2 and Llama shapes), then end to end with the best
# value against 0, and the streamed LM-head mode end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "rope or lm_head" --timeout 120 --timeout-method thread > gpurun_out/t_rope.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_rope.log; exit 1; }
tail -1 gpurun_out/t_rope.log
timeout -k 10 200 python -u -m pytest tests/test_model_gpu.py -x -q -k "streamed" --timeout 120 --timeout-method thread >> gpurun_out/t_rope.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_rope.log; exit 1; }
tail -1 gpurun_out/t_rope.log
timeout -k 10 300 python benchmarks/swiglu_bench.py --stagger-ab 0,1,2,3,4,6 --rounds 5 > gpurun_out/stag_gpt2.log 2>&1 || { tail -20 gpurun_out/stag_gpt2.log; exit 1; }
cat gpurun_out/stag_gpt2.log
timeout -k 10 300 python benchmarks/swiglu_bench.py --tokens 16384 --dim 2048 --ff 5632 --stagger-ab 0,1,2,3,4,6 --rounds 5 > gpurun_out/stag_llama.log 2>&1 || { tail -20 gpurun_out/stag_llama.log; exit 1; }
cat gpurun_out/stag_llama.log
best=$(python - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/stag_gpt2.log") if l.startswith("{")]
tot={}
for r in rows: tot[r["stagger"]]=tot.get(r["stagger"],0)+r["ms_median"]
print(min(tot,key=tot.get))
PY
)
echo best $best
for v in 0 $best 0 $best; do
  BPE_GPP_STAGGER=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_stag_$v.log 2>&1 || { tail -20 gpurun_out/bench_stag_$v.log; exit 1; }
  echo "stagger $v: $(tail -1 gpurun_out/bench_stag_$v.log)"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lm-head-mode streamed > gpurun_out/bench_streamed.log 2>&1 || { tail -20 gpurun_out/bench_streamed.log; exit 1; }
echo "streamed: $(tail -1 gpurun_out/bench_streamed.log)"
BPE_GPP_STAGGER=$best bash tools/gpu/prof_step.sh r3b > /dev/null 2>&1; head -30 gpurun_out/prof_r3b.md
