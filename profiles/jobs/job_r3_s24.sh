#!/usr/bin/env bash
# r03 s24: norm_apply with 16-B operand loads: bit-identity vs HEAD, layers, step A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
H=build/rev_head/_lib
L() { echo "OFLOW_LIB=build/$1/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/$1/_lib/liboflow_torch.so"; }
tools/gpu_job.sh \
 "120|s24_dump_new|TAG=new python -u tools/exp/enc_dump.py" \
 "120|s24_dump_head|TAG=head $(L rev_head) python -u tools/exp/enc_dump.py" \
 "60|s24_cmp|python tools/exp/enc_dump.py --compare new head; rm -f gpurun_out/enc_*.pt" \
 "120|s24_layers_new|python -u tools/exp/run_encoder_layers.py" \
 "120|s24_layers_head|$(L rev_head) python -u tools/exp/run_encoder_layers.py" \
 "120|s24_ab_new1|python -u tools/exp/step_ab.py" \
 "120|s24_ab_head1|$(L rev_head) python -u tools/exp/step_ab.py" \
 "120|s24_ab_new2|python -u tools/exp/step_ab.py" \
 "120|s24_ab_head2|$(L rev_head) python -u tools/exp/step_ab.py"
