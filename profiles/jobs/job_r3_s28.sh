#!/usr/bin/env bash
# r03 s28: the corr pyramid built per pair lane (RAFT.pyramid_lanes): bit-identity tests, in-process step A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|s28_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_raft.py" \
 "300|s28_ab|ATTRS='{\"one\": {\"pyramid_lanes\": false}, \"lanes\": {\"pyramid_lanes\": true}}' SAMPLES=8 python -u tools/exp/attr_ab.py"
