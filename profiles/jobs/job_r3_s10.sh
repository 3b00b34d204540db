#!/usr/bin/env bash
# r03 s10: high-priority fnet streams A/B; BN64 4-row default check
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|s10_ab_prio|SAMPLES=8 ATTRS='{\"base\": {}, \"prio\": {\"fnet_priority\": true}, \"base_\": {\"fnet_priority\": false}, \"prio_\": {\"fnet_priority\": true}}' python -u tools/exp/attr_ab.py" \
 "300|s10_ab_bn64|SAMPLES=6 ATTRS='{\"r4\": {}, \"r8\": {\"lib:oflow_exp_set_bn64_8row\": 1}, \"r4_\": {\"lib:oflow_exp_set_bn64_8row\": 0}}' python -u tools/exp/attr_ab.py"
