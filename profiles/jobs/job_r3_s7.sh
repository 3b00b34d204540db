#!/usr/bin/env bash
# r03 s7: pinned prefetch loads in conv_s32 (sched_barrier) A/B: convbench + encoder layers + step, vs no-pin / HEAD
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
L() { echo "OFLOW_LIB=build/$1/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/$1/_lib/liboflow_torch.so"; }
tools/gpu_job.sh \
 "120|s7_conv_pin|python -u tools/convbench.py" \
 "120|s7_conv_nopin|$(L nopin) python -u tools/convbench.py" \
 "120|s7_layers_pin|python -u tools/exp/run_encoder_layers.py" \
 "120|s7_layers_nopin|$(L nopin) python -u tools/exp/run_encoder_layers.py" \
 "120|s7_layers_s4row|$(L s4row) python -u tools/exp/run_encoder_layers.py" \
 "120|s7_ab_pin1|python -u tools/exp/step_ab.py" \
 "120|s7_ab_head1|$(L rev_head) python -u tools/exp/step_ab.py" \
 "120|s7_ab_s4row1|$(L s4row) python -u tools/exp/step_ab.py" \
 "120|s7_ab_pin2|python -u tools/exp/step_ab.py" \
 "120|s7_ab_head2|$(L rev_head) python -u tools/exp/step_ab.py" \
 "120|s7_ab_s4row2|$(L s4row) python -u tools/exp/step_ab.py" \
 "300|s7_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_raft.py tests/test_gpu_conv_s32.py tests/test_gpu_corr_convc1.py"
