#!/usr/bin/env bash
# r03 s17: conv weights register-staged two steps ahead: tests, convbench and step A/B vs HEAD
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
L() { echo "OFLOW_LIB=build/$1/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/$1/_lib/liboflow_torch.so"; }
tools/gpu_job.sh \
 "300|s17_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "200|s17_conv_new|python -u tools/convbench.py --no-lookup" \
 "200|s17_conv_head|$(L rev_head) python -u tools/convbench.py --no-lookup" \
 "120|s17_ab_new1|python -u tools/exp/step_ab.py" \
 "120|s17_ab_head1|$(L rev_head) python -u tools/exp/step_ab.py" \
 "120|s17_ab_new2|python -u tools/exp/step_ab.py" \
 "120|s17_ab_head2|$(L rev_head) python -u tools/exp/step_ab.py"
