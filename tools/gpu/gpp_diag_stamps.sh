# ping-pong main-loop diagnostics: per-tile stamps of the plain GEMMs in the normal stamps build and in DIAG builds
# (1 = no DMA in the loop, 2 = fragment reads only in phase 0, 3 = no MFMA); numerically wrong, timing only
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in stamps sd1 sd2 sd3; do
  echo "== variant $v"
  BPE_HIP_VARIANT=$v timeout -k 10 200 python benchmarks/gemm_stamps.py 2>&1 | grep -v amdgpu.ids | grep -A1 "qkv fwd\|w13 fwd plain" | grep -v "^--"
done
