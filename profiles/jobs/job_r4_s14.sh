#!/usr/bin/env bash
# register-direct weights (BREG): parity, per-layer micro-bench both ways, in-process step A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
  "240|r4s14_tests|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py" \
  "180|r4s14_cb_breg|python -u tools/convbench.py" \
  "180|r4s14_cb_lds|OFLOW_CONV_BREG=0 python -u tools/convbench.py" \
  "400|r4s14_ab|ATTRS='{\"lds\": {\"native:CONV_BREG\": false}, \"breg\": {\"native:CONV_BREG\": true}}' SAMPLES=8 python -u tools/exp/attr_ab.py"
