#!/usr/bin/env bash
# r04 s27: 256-channel register-direct workgroups (8 waves, one per CU) for GRU z|r and fh1 (hook oflow_exp_set_breg8w)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "240|r4s27_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py" \
 "120|r4s27_cb8w|python -u tools/convbench.py --no-lookup --breg8w" \
 "120|r4s27_cb|python -u tools/convbench.py --no-lookup" \
 "500|r4s27_ab|ATTRS='{\"w4\": {\"lib:oflow_exp_set_breg8w\": 0}, \"w8\": {\"lib:oflow_exp_set_breg8w\": 1}}' SAMPLES=10 python -u tools/exp/attr_ab.py"
