#!/usr/bin/env bash
# r06 s13: the whole GPU suite on the tree with oflow_conv_s32_ex5 (split-K off in the forward), smoke
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "900|r6s13_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests -rf" \
 "200|r6s13_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'"
