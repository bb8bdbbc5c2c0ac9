cd $GRAFT_REPO_ROOT
for d in 0 16 2 4 8 0 16; do
  echo "diag=$d $(BPE_HIP_VARIANT=diag BPE_FA_DIAG=$d timeout -k 5 100 python -u benchmarks/attn_bench.py --batch 128 --iters 20 2>/dev/null | tail -1)"
done
