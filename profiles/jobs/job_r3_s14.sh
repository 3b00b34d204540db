#!/usr/bin/env bash
# r03 s14: update-block conv ablations at the lane shape (4 pairs) and 8 pairs
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
L() { echo "OFLOW_LIB=build/$1/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/$1/_lib/liboflow_torch.so"; }
tools/gpu_job.sh \
 "200|s14_upd_abl4|$(L abl) python -u tools/convbench.py --no-lookup --ablate --shape-batch 4" \
 "200|s14_upd_abl8|$(L abl) python -u tools/convbench.py --no-lookup --ablate"
