#!/usr/bin/env bash
# r03 s30: flow head output conv with split K: tests, in-process step A/B over the slice count
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|s30_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "400|s30_ab|ATTRS='{\"k1\": {\"mod:model.update.FH2_KSPLIT\": 1}, \"k2\": {\"mod:model.update.FH2_KSPLIT\": 2}, \"k4\": {\"mod:model.update.FH2_KSPLIT\": 4}, \"k8\": {\"mod:model.update.FH2_KSPLIT\": 8}}' SAMPLES=8 python -u tools/exp/attr_ab.py"
