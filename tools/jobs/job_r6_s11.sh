#!/usr/bin/env bash
# r06 s11: which topology crashes on PyTorch's bundled HIP runtime: lane 1's side stream alone (nested fork), then the
# full topology without AMD logging (exit status recorded)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TL=$(python -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
mkdir -p /tmp/torchrt && ln -sf "$TL/libamdhip64.so" /tmp/torchrt/libamdhip64.so.7
RT="/tmp/torchrt:$TL"
tools/gpu_job.sh \
 "60|r6s11_torchrt_lane1side|LD_LIBRARY_PATH=$RT ./build/exp/capture_fork_repro lane1side 12 2" \
 "60|r6s11_torchrt_full|LD_LIBRARY_PATH=$RT ./build/exp/capture_fork_repro full 12 2"
