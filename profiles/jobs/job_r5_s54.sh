#!/usr/bin/env bash
# r05 s54: the tiled flow head writing the next update's flow channels (no flow_prep per update): tests, then graph
# bench A/B against OFLOW_FLOW_FROM_HEAD=0, alternated
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "600|r5s54_test|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "300|r5s54_new1|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s54_old1|OFLOW_FLOW_FROM_HEAD=0 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s54_new2|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s54_old2|OFLOW_FLOW_FROM_HEAD=0 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s54_new3|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s54_old3|OFLOW_FLOW_FROM_HEAD=0 python -u bench.py --no-cpu-baseline --no-step-flops"
