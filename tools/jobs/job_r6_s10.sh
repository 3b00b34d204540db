#!/usr/bin/env bash
# r06 s10: the HIP-only capture repro against the HIP runtime PyTorch ships (torch/lib/libamdhip64.so, soname
# libamdhip64.so.7: the one every torch process -- and therefore liboflow_hip.so inside it -- runs on) instead of
# /opt/rocm-7.2's (the repro's RUNPATH). The file is exposed as libamdhip64.so.7 in a scratch directory.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TL=$(python -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
mkdir -p /tmp/torchrt && ln -sf "$TL/libamdhip64.so" /tmp/torchrt/libamdhip64.so.7
RT="/tmp/torchrt:$TL"
tools/gpu_job.sh \
 "60|r6s10_torchrt_ldd|LD_LIBRARY_PATH=$RT ldd ./build/exp/capture_fork_repro | grep amdhip" \
 "60|r6s10_torchrt_nolaneside|LD_LIBRARY_PATH=$RT ./build/exp/capture_fork_repro nolaneside 12 2" \
 "60|r6s10_torchrt_lane0side|LD_LIBRARY_PATH=$RT ./build/exp/capture_fork_repro lane0side 12 2" \
 "60|r6s10_torchrt_full|LD_LIBRARY_PATH=$RT AMD_LOG_LEVEL=3 ./build/exp/capture_fork_repro full 12 2 2>&1 | grep -E 'EndCapture|EmptyNode|RESULT|HIP error|captured|eager'"
