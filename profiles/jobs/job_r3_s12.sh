#!/usr/bin/env bash
# r03 s12: encoder conv ablations (stem, layer1)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|s12_enc_abl|OFLOW_LIB=build/abl/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/abl/_lib/liboflow_torch.so python -u tools/exp/run_enc_abl.py"
