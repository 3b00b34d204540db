#!/usr/bin/env bash
# Build the fused lookup + convc1 experiment variants (tools/exp/corr_convc1_variants.hip) into build/exp/libc1var.so
set -euo pipefail
REPO="$(cd "$(dirname "$0")/../.." && pwd)"
mkdir -p "$REPO/build/exp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I"$REPO/include" -fno-slp-vectorize -fno-vectorize \
  "$REPO/tools/exp/corr_convc1_variants.hip" -o "$REPO/build/exp/libc1var.so"
echo "$REPO/build/exp/libc1var.so"
