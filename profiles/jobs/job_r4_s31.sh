#!/usr/bin/env bash
# r04 s31: 64-channel register-direct blocks (CONV_BREG64) with the motion conv / fh1 split into 64-channel blocks
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "700|r4s31_ab|ATTRS='{\"base\": {\"native:CONV_BREG64\": false, \"bn:mo\": 128, \"bn:fh1\": 128}, \"b64\": {\"native:CONV_BREG64\": true, \"bn:mo\": 128, \"bn:fh1\": 128}, \"b64_mo\": {\"native:CONV_BREG64\": true, \"bn:mo\": 64, \"bn:fh1\": 128}, \"b64_mo_fh1\": {\"native:CONV_BREG64\": true, \"bn:mo\": 64, \"bn:fh1\": 64}}' SAMPLES=8 python -u tools/exp/attr_ab.py"
