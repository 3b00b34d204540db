#!/usr/bin/env bash
# r04 s26: 256-channel register-direct workgroups (8 waves, one per CU) for GRU z|r and fh1 (hook oflow_exp_set_breg256)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "240|r4s26_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py" \
 "120|r4s26_cb256|python -u tools/convbench.py --no-lookup --breg256" \
 "120|r4s26_cb|python -u tools/convbench.py --no-lookup" \
 "500|r4s26_ab|ATTRS='{\"b128\": {\"lib:oflow_exp_set_breg256\": 0}, \"b256\": {\"lib:oflow_exp_set_breg256\": 1}}' SAMPLES=10 python -u tools/exp/attr_ab.py"
