#!/usr/bin/env bash
# r03 s35: norm statistics finalize with 16 partials in flight (build/rev_ns16) vs the tree: encoder bit-identity,
# tests on the new library, step A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
L() { echo "OFLOW_LIB=build/$1/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/$1/_lib/liboflow_torch.so"; }
tools/gpu_job.sh \
 "120|s35_dump_new|TAG=new $(L rev_ns16) python -u tools/exp/enc_dump.py" \
 "120|s35_dump_head|TAG=head python -u tools/exp/enc_dump.py" \
 "60|s35_cmp|python tools/exp/enc_dump.py --compare new head; rm -f gpurun_out/enc_*.pt" \
 "300|s35_pytest|$(L rev_ns16) python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "120|s35_ab_new1|$(L rev_ns16) python -u tools/exp/step_ab.py" \
 "120|s35_ab_head1|python -u tools/exp/step_ab.py" \
 "120|s35_ab_new2|$(L rev_ns16) python -u tools/exp/step_ab.py" \
 "120|s35_ab_head2|python -u tools/exp/step_ab.py"
