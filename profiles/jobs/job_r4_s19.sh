#!/usr/bin/env bash
# r04 s19: register-direct weights for the 64-channel 3x3 blocks as 2 x 2 waves (CONV_BREG64)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "240|r4s19_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py" \
 "120|r4s19_cb64|OFLOW_CONV_BREG64=1 python -u tools/convbench.py --no-lookup" \
 "120|r4s19_cb|python -u tools/convbench.py --no-lookup" \
 "400|r4s19_ab|ATTRS='{\"lds64\": {\"native:CONV_BREG64\": false}, \"breg64\": {\"native:CONV_BREG64\": true}}' SAMPLES=10 python -u tools/exp/attr_ab.py"
