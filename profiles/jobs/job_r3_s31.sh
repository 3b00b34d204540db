#!/usr/bin/env bash
# r03 s31: BN 128 convs on 8-row tiles with 8 waves (one workgroup per CU): in-process step A/B (bit-identity reported)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "400|s31_ab|ATTRS='{\"w4\": {\"lib:oflow_exp_set_bn128_8w\": 0}, \"w8\": {\"lib:oflow_exp_set_bn128_8w\": 1}}' SAMPLES=8 python -u tools/exp/attr_ab.py"
