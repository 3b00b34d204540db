#!/usr/bin/env bash
# r04 s30: staggered start of register-direct workgroups (hook oflow_exp_set_conv_stagger: x 1024 cycles)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "600|r4s30_ab|ATTRS='{\"s0\": {\"lib:oflow_exp_set_conv_stagger\": 0}, \"s2\": {\"lib:oflow_exp_set_conv_stagger\": 2}, \"s4\": {\"lib:oflow_exp_set_conv_stagger\": 4}, \"s8\": {\"lib:oflow_exp_set_conv_stagger\": 8}}' SAMPLES=8 python -u tools/exp/attr_ab.py"
