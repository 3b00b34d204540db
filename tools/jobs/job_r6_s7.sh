#!/usr/bin/env bash
# r06 s7: the HIP-only capture repro at torch's node count (2 kernels per op) and at 4x the iterations
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "60|r6s7_hip_full_x2|AMD_LOG_LEVEL=3 ./build/exp/capture_fork_repro full 12 2 2>&1 | grep -E 'EndCapture|EmptyNode|RESULT|error'" \
 "60|r6s7_hip_full_i48|AMD_LOG_LEVEL=3 ./build/exp/capture_fork_repro full 48 1 2>&1 | grep -E 'EndCapture|EmptyNode|RESULT|error'" \
 "60|r6s7_hip_full_i48x2|AMD_LOG_LEVEL=3 ./build/exp/capture_fork_repro full 48 2 2>&1 | grep -E 'EndCapture|EmptyNode|RESULT|error'"
