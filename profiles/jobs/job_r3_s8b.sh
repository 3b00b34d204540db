#!/usr/bin/env bash
# r03 s8b: in-process step A/B of the encoder changes (8-row instance-norm tiles, batched stem window loads) and of
# non-temporal pyramid stores
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|s8b_ab_enc|SAMPLES=8 ATTRS='{\"new\": {}, \"stats4\": {\"lib:oflow_exp_set_stats_8row\": 0}, \"stemloop\": {\"lib:oflow_exp_set_conv_flags\": 1}, \"both_old\": {\"lib:oflow_exp_set_stats_8row\": 0, \"lib:oflow_exp_set_conv_flags\": 1}, \"new_\": {\"lib:oflow_exp_set_stats_8row\": 1, \"lib:oflow_exp_set_conv_flags\": 0}}' python -u tools/exp/attr_ab.py" \
 "300|s8b_ab_nt|SAMPLES=8 ATTRS='{\"plain\": {}, \"nt\": {\"lib:oflow_exp_set_pyramid_nt\": 1}, \"plain_\": {\"lib:oflow_exp_set_pyramid_nt\": 0}}' python -u tools/exp/attr_ab.py"
