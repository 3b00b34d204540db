#!/usr/bin/env bash
# r05 s33: the LDS-tiled (512 threads, 4 channel quarters) fp32-FMA flow-head output conv: its tests, then whole-step A/B against the split conv
# (OFLOW_FLOW_HEAD_MODE=tiled vs the default conv), same library, and the RAFT parity tests in tiled mode
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s33_test|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py -k flow_head2" \
 "200|r5s33_conv1|python -u tools/exp/step_ab.py" \
 "200|r5s33_tiled1|OFLOW_FLOW_HEAD_MODE=tiled python -u tools/exp/step_ab.py" \
 "200|r5s33_conv2|python -u tools/exp/step_ab.py" \
 "200|r5s33_tiled2|OFLOW_FLOW_HEAD_MODE=tiled python -u tools/exp/step_ab.py" \
 "200|r5s33_conv3|python -u tools/exp/step_ab.py" \
 "200|r5s33_tiled3|OFLOW_FLOW_HEAD_MODE=tiled python -u tools/exp/step_ab.py" \
 "600|r5s33_parity|OFLOW_FLOW_HEAD_MODE=tiled python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_raft.py"
