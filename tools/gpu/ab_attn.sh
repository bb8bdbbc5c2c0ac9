# Same-box A/B of the attention microbenchmark: bash tools/gpu/ab_attn.sh "<bench args>" "VAR=a" "VAR=b" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
args=$1; shift
for rep in 1 2; do
  for spec in "$@"; do
    line=$(env $spec timeout -k 10 120 python3 -u benchmarks/attn_bench.py $args 2>/dev/null | tail -1)
    rc=$?
    echo "[$spec] $line"
    [ $rc -ne 0 ] && echo "failed rc=$rc" && exit 1
  done
done
exit 0
