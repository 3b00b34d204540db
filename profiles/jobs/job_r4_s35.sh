#!/usr/bin/env bash
# r04 s35: one-kernel input scaling (oflow_normalize_images_f32) vs the ATen elementwise form
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r4s35_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_raft.py tests/test_gpu_ops.py" \
 "500|r4s35_ab|ATTRS='{\"aten\": {\"mod:model.raft.NATIVE_NORMALIZE\": false}, \"native\": {\"mod:model.raft.NATIVE_NORMALIZE\": true}}' SAMPLES=10 python -u tools/exp/attr_ab.py"
