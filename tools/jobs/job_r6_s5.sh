#!/usr/bin/env bash
# r06 s5: the crashing torch topology captured by raw hipStreamBeginCapture/EndCapture (ctypes), then the torch.cuda.graph
# capture under AMD_LOG_LEVEL=3 (last: it ends the job)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "120|r6s5_torch_raw|python -X faulthandler -u tools/exp/capture_fork_torch_repro.py raw" \
 "120|r6s5_torch_ops_log|AMD_LOG_LEVEL=3 python -X faulthandler -u tools/exp/capture_fork_torch_repro.py ops > gpurun_out/r6s5_ops_amdlog.txt 2>&1"
