#!/usr/bin/env bash
# r06 s4: bisect the torch-level capture crash (tools/exp/capture_fork_torch_repro.py ops crashes, the HIP repro does
# not): without the lanes' side streams, events kept alive, raw hipStreamBeginCapture through ctypes; then the crashing
# mode under AMD_LOG_LEVEL=3 (last: it ends the job)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "120|r6s4_torch_noside|python -X faulthandler -u tools/exp/capture_fork_torch_repro.py noside" \
 "120|r6s4_torch_keep|python -X faulthandler -u tools/exp/capture_fork_torch_repro.py keep" \
 "120|r6s4_torch_raw|python -X faulthandler -u tools/exp/capture_fork_torch_repro.py raw" \
 "120|r6s4_torch_ops_log|AMD_LOG_LEVEL=3 python -X faulthandler -u tools/exp/capture_fork_torch_repro.py ops > gpurun_out/r6s4_ops_amdlog.txt 2>&1"
