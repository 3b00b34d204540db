#!/usr/bin/env bash
# BREG for 64-channel 3x3 blocks (two-wave workgroups) and with instance-norm partials; hardware GRU gates default
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-events --no-step-flops"
tools/gpu_job.sh \
  "300|r4s16_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py tests/test_gpu_corr_convc1.py" \
  "120|r4s16_cb|python -u tools/convbench.py" \
  "400|r4s16_ab|ATTRS='{\"lds\": {\"native:CONV_BREG\": false}, \"breg\": {\"native:CONV_BREG\": true}}' SAMPLES=8 python -u tools/exp/attr_ab.py" \
  "120|r4s16_b1|$B" "120|r4s16_b2|$B"
