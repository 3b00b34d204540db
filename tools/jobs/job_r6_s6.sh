#!/usr/bin/env bash
# r06 s6: the crashing torch-level capture under AMD_LOG_LEVEL=3 (the stream / event / capture calls before the crash)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 env AMD_LOG_LEVEL=3 python -X faulthandler -u tools/exp/capture_fork_torch_repro.py ops > gpurun_out/r6s6_ops_amdlog.txt 2>&1
rc=$?
grep -v -E "hipGetDevice|hipGetLastError|hipPeekAtLastError|hipDevicePrimaryCtxGetState|hipModuleLaunchKernel|hipLaunchKernel|hipExtLaunch|KernelNode|hipGetDeviceCount|hipDeviceGetAttribute|hipStreamGetCaptureInfo|hipSetDevice|hipPointerGetAttribute|ShaderName|hipFuncGetAttributes" gpurun_out/r6s6_ops_amdlog.txt > gpurun_out/r6s6_ops_amdlog_filtered.txt
gzip -f gpurun_out/r6s6_ops_amdlog.txt
exit $rc
