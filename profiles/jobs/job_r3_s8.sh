#!/usr/bin/env bash
# r03 s8: pyramid levels 2-3 staged + NT store A/B; pyramid tests; step A/B vs HEAD
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
L() { echo "OFLOW_LIB=build/$1/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/$1/_lib/liboflow_torch.so"; }
tools/gpu_job.sh \
 "300|s8_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pyramid_s32.py tests/test_gpu_parity.py tests/test_gpu_raft.py" \
 "120|s8_pyr_ab|python -u tools/exp/run_pyr_ab.py" \
 "120|s8_kbench_new|python -u tools/kbench.py" \
 "120|s8_kbench_head|$(L rev_head) python -u tools/kbench.py" \
 "120|s8_ab_new1|python -u tools/exp/step_ab.py" \
 "120|s8_ab_head1|$(L rev_head) python -u tools/exp/step_ab.py" \
 "120|s8_ab_new2|python -u tools/exp/step_ab.py" \
 "120|s8_ab_head2|$(L rev_head) python -u tools/exp/step_ab.py"
