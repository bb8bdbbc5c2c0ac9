#!/bin/bash
# Build the HIP library of another git revision as an A/B variant: bpe_transformer/ops/_bpe_hip_<name>.so,
# selected at run time with BPE_HIP_VARIANT=<name> (same process tree, same box as the in-tree library).
# usage: tools/ab_build.sh <rev> <name>
set -e
cd "$(dirname "$0")/.."
rev=${1:?revision}; name=${2:?variant name}
tmp=$(mktemp -d)
git archive "$rev" bpe_transformer/ops/csrc | tar -x -C "$tmp"
python -m bpe_transformer.ops.build --variant "$name" --src "$tmp/bpe_transformer/ops/csrc"
rm -rf "$tmp"
