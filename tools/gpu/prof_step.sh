# Kernel-trace profile of the bench.py default step (timed steps only) -> markdown summary.
# usage (GPU box): bash tools/gpu/prof_step.sh <tag> [bench args...]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag=${1:-step}; shift || true
out=gpurun_out/prof_$tag
rm -rf $out
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out -o prof -- python3 bench.py --steps 5 --warmup 3 "$@" > gpurun_out/prof_$tag.log 2>&1
csv=$(find $out -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$csv" --steps 5 --warmup 3 --title "$tag" > gpurun_out/prof_$tag.md
rm -rf $out
cat gpurun_out/prof_$tag.md | head -40
