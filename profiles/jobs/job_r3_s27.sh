#!/usr/bin/env bash
# r03 s27: barrier-free stem (per-wave A fragments from the window, weights resident): bit-identity vs HEAD, tests,
# ablation, step A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
L() { echo "OFLOW_LIB=build/$1/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/$1/_lib/liboflow_torch.so"; }
tools/gpu_job.sh \
 "120|s27_dump_new|TAG=new python -u tools/exp/enc_dump.py" \
 "120|s27_dump_head|TAG=head $(L rev_head) python -u tools/exp/enc_dump.py" \
 "60|s27_cmp|python tools/exp/enc_dump.py --compare new head; rm -f gpurun_out/enc_*.pt" \
 "700|s27_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
 "120|s27_ab_new1|python -u tools/exp/step_ab.py" \
 "120|s27_ab_head1|$(L rev_head) python -u tools/exp/step_ab.py" \
 "120|s27_ab_new2|python -u tools/exp/step_ab.py" \
 "120|s27_ab_head2|$(L rev_head) python -u tools/exp/step_ab.py"
