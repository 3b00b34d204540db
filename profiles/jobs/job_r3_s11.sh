#!/usr/bin/env bash
# r03 s11: smaller update-conv blocks in the step (GRU 64-channel blocks, motion conv / fh1 BN 64)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "400|s11_ab_blocks|SAMPLES=6 ATTRS='{\"base\": {\"lib:oflow_exp_set_gru_bn64\": 0, \"bn:mo\": 128, \"bn:fh1\": 128}, \"gru64\": {\"lib:oflow_exp_set_gru_bn64\": 1, \"bn:mo\": 128, \"bn:fh1\": 128}, \"mo64\": {\"lib:oflow_exp_set_gru_bn64\": 0, \"bn:mo\": 64, \"bn:fh1\": 128}, \"fh64\": {\"lib:oflow_exp_set_gru_bn64\": 0, \"bn:mo\": 128, \"bn:fh1\": 64}, \"all64\": {\"lib:oflow_exp_set_gru_bn64\": 1, \"bn:mo\": 64, \"bn:fh1\": 64}}' python -u tools/exp/attr_ab.py"
