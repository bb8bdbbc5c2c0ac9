# A/B bench.py under environment settings: bash tools/gpu/ab_env.sh "VAR=1 VAR2=x" "VAR=0" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for spec in "$@"; do
  line=$(env $spec timeout -k 10 240 python3 -u bench.py 2>/dev/null | grep '"metric"')
  rc=$?
  echo "[$spec] $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])' 2>/dev/null)"
  [ $rc -ne 0 ] && echo "failed rc=$rc" && exit 1
done
exit 0
