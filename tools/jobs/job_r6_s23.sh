#!/usr/bin/env bash
# r06 s23: API lookup with non-temporal output stores vs HEAD (OFLOW_LIB=build/ab_old), the bench's lookup and warp
# legs alone (tools/exp/run_api_legs.py), alternated in separate processes on one box
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
R="python3 tools/exp/run_api_legs.py"
tools/gpu_job.sh \
 "300|r6s23_gpu_lookup|python3 -u -m pytest tests/test_gpu_parity.py -x -q -k lookup --timeout 120 --timeout-method thread" \
 "120|r6s23_old1|OFLOW_LIB=build/ab_old/liboflow_hip.so $R" \
 "120|r6s23_new1|$R" \
 "120|r6s23_old2|OFLOW_LIB=build/ab_old/liboflow_hip.so $R" \
 "120|r6s23_new2|$R" \
 "120|r6s23_old3|OFLOW_LIB=build/ab_old/liboflow_hip.so $R" \
 "120|r6s23_new3|$R"
