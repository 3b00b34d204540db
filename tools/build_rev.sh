#!/usr/bin/env bash
# Build liboflow_hip.so + liboflow_torch.so of a git revision into build/rev_<name>/_lib (for in-process or
# back-to-back A/B runs on the GPU box: OFLOW_LIB / OFLOW_OPS_LIB point the package at them).
# usage: tools/build_rev.sh <git-rev> [name]
set -euo pipefail
REPO="$(cd "$(dirname "$0")/.." && pwd)"
rev="$1"; name="${2:-$1}"
dst="$REPO/build/rev_$name"
rm -rf "$dst"; mkdir -p "$dst"
git -C "$REPO" archive "$rev" torch-optical-flow_amd/csrc include | tar -x -C "$dst"
make -C "$dst/torch-optical-flow_amd/csrc" -j8 OUTDIR="$dst/_lib" >/dev/null
echo "$dst/_lib"
