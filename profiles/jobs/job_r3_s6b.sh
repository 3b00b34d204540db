#!/usr/bin/env bash
# r03 s6b: stem window loads batched + 8-row tiles for instance-norm convs: bit-identity vs HEAD, per-layer timing, step A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
H=build/rev_head/_lib
tools/gpu_job.sh \
 "120|s6b_dump_new|TAG=new python -u tools/exp/enc_dump.py" \
 "120|s6b_dump_head|TAG=head OFLOW_LIB=$H/liboflow_hip.so OFLOW_OPS_LIB=$H/liboflow_torch.so python -u tools/exp/enc_dump.py" \
 "60|s6b_cmp|python tools/exp/enc_dump.py --compare new head; rm -f gpurun_out/enc_*.pt" \
 "120|s6b_layers_new|python -u tools/exp/run_encoder_layers.py" \
 "120|s6b_layers_head|OFLOW_LIB=$H/liboflow_hip.so OFLOW_OPS_LIB=$H/liboflow_torch.so python -u tools/exp/run_encoder_layers.py" \
 "120|s6b_ab_new1|python -u tools/exp/step_ab.py" \
 "120|s6b_ab_head1|OFLOW_LIB=$H/liboflow_hip.so OFLOW_OPS_LIB=$H/liboflow_torch.so python -u tools/exp/step_ab.py" \
 "120|s6b_ab_new2|python -u tools/exp/step_ab.py" \
 "120|s6b_ab_head2|OFLOW_LIB=$H/liboflow_hip.so OFLOW_OPS_LIB=$H/liboflow_torch.so python -u tools/exp/step_ab.py" \
 "300|s6b_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_raft.py tests/test_gpu_conv_s32.py"
