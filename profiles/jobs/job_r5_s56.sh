#!/usr/bin/env bash
# r05 s56: graph capture with the first lane's side stream kept (OFLOW_CAPTURE_SIDE=lane0: a single-level fork from the
# capture stream) and the second lane inline: bench A/B against the default, then the graph tests in that mode last
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s56_base1|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s56_lane0a|OFLOW_CAPTURE_SIDE=lane0 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s56_base2|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s56_lane0b|OFLOW_CAPTURE_SIDE=lane0 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s56_test|OFLOW_CAPTURE_SIDE=lane0 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_raft.py -k graphed"
