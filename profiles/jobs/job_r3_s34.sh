#!/usr/bin/env bash
# r03 s34: norm statistics finalize with 16 partials in flight: bit-identity of the encoders vs HEAD, tests, step A/B,
# kernel times
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
L() { echo "OFLOW_LIB=build/$1/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/$1/_lib/liboflow_torch.so"; }
tools/gpu_job.sh \
 "120|s34_dump_new|TAG=new python -u tools/exp/enc_dump.py" \
 "120|s34_dump_head|TAG=head $(L rev_head) python -u tools/exp/enc_dump.py" \
 "60|s34_cmp|python tools/exp/enc_dump.py --compare new head; rm -f gpurun_out/enc_*.pt" \
 "300|s34_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "120|s34_ab_new1|python -u tools/exp/step_ab.py" \
 "120|s34_ab_head1|$(L rev_head) python -u tools/exp/step_ab.py" \
 "120|s34_ab_new2|python -u tools/exp/step_ab.py" \
 "120|s34_ab_head2|$(L rev_head) python -u tools/exp/step_ab.py" \
 "200|s34_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s34_prof -o run -- python3 tools/exp/step_ab.py" \
 "60|s34_stats|S=\$(find gpurun_out/s34_prof -name '*kernel_stats.csv' | head -1); grep -E 'norm_stats|norm_apply' \$S; rm -rf gpurun_out/s34_prof"
