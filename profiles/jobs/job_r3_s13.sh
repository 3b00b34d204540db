#!/usr/bin/env bash
# r03 s13: instance-norm partials from the accumulators: tests, ablation, step A/B vs HEAD
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
L() { echo "OFLOW_LIB=build/$1/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/$1/_lib/liboflow_torch.so"; }
tools/gpu_job.sh \
 "300|s13_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "200|s13_enc_abl|$(L abl) python -u tools/exp/run_enc_abl.py" \
 "120|s13_layers|python -u tools/exp/run_encoder_layers.py" \
 "120|s13_ab_new1|python -u tools/exp/step_ab.py" \
 "120|s13_ab_head1|$(L rev_head) python -u tools/exp/step_ab.py" \
 "120|s13_ab_new2|python -u tools/exp/step_ab.py" \
 "120|s13_ab_head2|$(L rev_head) python -u tools/exp/step_ab.py"
