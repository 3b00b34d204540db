#!/usr/bin/env bash
# r06 s9: warp strip-kernel variants A/B (1 = r03 kernel, 2 = flow prefetched kSD steps ahead, 3 = 2 + non-temporal
# output stores), bit-identity across them; then the HIP-only capture repro with hipSetDevice before every operation
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "180|r6s9_warp_ab|HOOK=oflow_exp_set_warp_strip CPW=1,2,3 python -u tools/exp/run_warp_ab.py" \
 "60|r6s9_hip_nolaneside_setdev|./build/exp/capture_fork_repro nolaneside 12 2 1" \
 "60|r6s9_hip_lane0side_setdev|./build/exp/capture_fork_repro lane0side 12 2 1" \
 "60|r6s9_hip_full_setdev|./build/exp/capture_fork_repro full 12 2 1"
