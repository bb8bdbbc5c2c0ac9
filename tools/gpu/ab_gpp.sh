# Same-box A/B of the ping-pong GEMM microbenchmark: bash tools/gpu/ab_gpp.sh "<bench args>" "VAR=a" "VAR=b" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
args=$1; shift
for rep in 1 2; do
  for spec in "$@"; do
    out=$(env $spec timeout -k 10 150 python3 -u benchmarks/gemm_pp_bench.py $args 2>/dev/null)
    rc=$?
    echo "[$spec] $(echo "$out" | python3 -c '
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d["name"], d.get("fwd_tf"), d.get("dX_tf"), d.get("dW_tf"), end=" | ")')"
    [ $rc -ne 0 ] && echo "failed rc=$rc" && exit 1
  done
done
exit 0
