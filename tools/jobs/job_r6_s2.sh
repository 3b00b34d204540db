#!/usr/bin/env bash
# r06 s2: HIP-only reduction of the two-lane capture crash (tools/exp/capture_fork_repro.hip), one process per
# topology, the configuration that crashes under torch last
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "60|r6s2_nolaneside|./build/exp/capture_fork_repro nolaneside" \
 "60|r6s2_lane0side|./build/exp/capture_fork_repro lane0side" \
 "60|r6s2_lane1side|./build/exp/capture_fork_repro lane1side" \
 "60|r6s2_keepevents|./build/exp/capture_fork_repro keepevents" \
 "60|r6s2_full|./build/exp/capture_fork_repro full"
