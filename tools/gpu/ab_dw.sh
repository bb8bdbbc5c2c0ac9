# Same-box A/B of the 256-tile dW GEMM variants: bash tools/gpu/ab_dw.sh 0 4 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for rep in 1 2; do
  for v in "$@"; do
    echo "[variant $v] $(BPE_G256_VARIANT=$v timeout -k 10 150 python3 -u benchmarks/gemm_dw.py 2>/dev/null | tail -1)"
  done
done
