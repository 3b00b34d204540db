#!/usr/bin/env bash
# r04 s23: register-direct 32-channel blocks (flow head output conv, CONV_BREG32) and 64-channel (CONV_BREG64) in the step
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "240|r4s23_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py" \
 "120|r4s23_cb32|OFLOW_CONV_BREG32=1 python -u tools/convbench.py --no-lookup" \
 "120|r4s23_cb|python -u tools/convbench.py --no-lookup" \
 "500|r4s23_ab|ATTRS='{\"base\": {\"native:CONV_BREG32\": false, \"native:CONV_BREG64\": false}, \"b32\": {\"native:CONV_BREG32\": true, \"native:CONV_BREG64\": false}, \"b32_64\": {\"native:CONV_BREG32\": true, \"native:CONV_BREG64\": true}}' SAMPLES=10 python -u tools/exp/attr_ab.py"
