#!/usr/bin/env bash
# r05 s48: the lanes' side streams under graph capture, pre-joined to the capture stream (OFLOW_CAPTURE_SIDE=1): the
# two-lane graph test first, then the graph bench against the default capture (no side streams). The side-stream
# capture crashed (segfault in capture_end) before the pre-join: its steps come last, so a crash ends the job there.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s48_base1|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s48_side_test|OFLOW_CAPTURE_SIDE=1 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_raft.py -k graphed" \
 "300|r5s48_side1|OFLOW_CAPTURE_SIDE=1 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s48_base2|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s48_side2|OFLOW_CAPTURE_SIDE=1 python -u bench.py --no-cpu-baseline --no-step-flops"
