#!/usr/bin/env bash
# r06 s3: the capture topology through torch (tools/exp/capture_fork_torch_repro.py): in-place ops, side-stream
# allocations, allocations everywhere; the HIP repro's end-capture log first
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "60|r6s3_hip_full_log|AMD_LOG_LEVEL=3 ./build/exp/capture_fork_repro full 2>&1 | grep -E 'EndCapture|EmptyNode|RESULT'" \
 "120|r6s3_torch_ops|python -X faulthandler -u tools/exp/capture_fork_torch_repro.py ops" \
 "120|r6s3_torch_lanealloc|python -X faulthandler -u tools/exp/capture_fork_torch_repro.py lanealloc" \
 "120|r6s3_torch_alloc|python -X faulthandler -u tools/exp/capture_fork_torch_repro.py alloc"
