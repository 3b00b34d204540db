#!/usr/bin/env bash
# r03 s29: per-lane pyramid, concurrent vs serialised (lane 1's after lane 0's): step A/B; tests with the rebuilt lib
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|s29_ab|ATTRS='{\"one\": {\"pyramid_lanes\": false}, \"lanes\": {\"pyramid_lanes\": true}, \"serial\": {\"pyramid_lanes\": \"serial\"}}' SAMPLES=8 python -u tools/exp/attr_ab.py" \
 "300|s29_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_raft.py"
