#!/usr/bin/env bash
# r04 s34: LDS-tiled flow_prep vs the per-thread form: bit-identity tests, step in-process A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r4s34_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "500|r4s34_ab|ATTRS='{\"untiled\": {\"lib:oflow_exp_set_flow_prep_untiled\": 1}, \"tiled\": {\"lib:oflow_exp_set_flow_prep_untiled\": 0}}' SAMPLES=10 python -u tools/exp/attr_ab.py"
