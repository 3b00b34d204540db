#!/usr/bin/env bash
# r06 s8: the HIP-only capture repro with hipSetDevice(0) before every operation (torch calls it 1316 times during the
# crashing capture): topology without the lanes' side streams first, then the full one
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "60|r6s8_hip_nolaneside_setdev|./build/exp/capture_fork_repro nolaneside 12 2 1" \
 "60|r6s8_hip_lane0side_setdev|./build/exp/capture_fork_repro lane0side 12 2 1" \
 "60|r6s8_hip_full_setdev|./build/exp/capture_fork_repro full 12 2 1"
