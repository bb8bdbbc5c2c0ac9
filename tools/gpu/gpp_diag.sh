# Ping-pong GEMM timing diagnostics (BPE_GPP_DIAG, variant library built with -DBPE_GPP_DIAG as "gdiag")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for d in 0 1 5 0 1 5; do
  echo "diag=$d $(BPE_HIP_VARIANT=gdiag BPE_GPP_DIAG=$d timeout -k 5 120 python -u benchmarks/gemm_pp_bench.py --quick --tokens ${TOKENS:-131072} 2>/dev/null | tr '\n' ' ')"
done
