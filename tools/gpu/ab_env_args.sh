# A/B bench.py under environment settings with extra bench args:
#   bash tools/gpu/ab_env_args.sh "<bench args>" "VAR=1" "VAR=0" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
args=$1; shift
for spec in "$@"; do
  line=$(env $spec timeout -k 10 300 python3 -u bench.py $args 2>/dev/null | grep '"metric"')
  rc=$?
  echo "[$spec] $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])' 2>/dev/null)"
  [ $rc -ne 0 ] && echo "failed rc=$rc" && exit 1
done
exit 0
