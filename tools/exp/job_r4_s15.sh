#!/usr/bin/env bash
# BREG with padded halo rows (immediate-offset A reads); hardware-exp2 GRU gates (conv flag 256)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
  "240|r4s15_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
  "180|r4s15_cb_breg|python -u tools/convbench.py" \
  "180|r4s15_cb_hw|python -u tools/convbench.py --conv-flags 256" \
  "400|r4s15_ab|ATTRS='{\"lds\": {\"native:CONV_BREG\": false, \"lib:oflow_exp_set_conv_flags\": 0}, \"breg\": {\"native:CONV_BREG\": true, \"lib:oflow_exp_set_conv_flags\": 0}, \"breg_hw\": {\"native:CONV_BREG\": true, \"lib:oflow_exp_set_conv_flags\": 256}}' SAMPLES=8 python -u tools/exp/attr_ab.py"
