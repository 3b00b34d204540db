#!/usr/bin/env bash
# padded operand rows (all conv variants; BREG immediate-offset A reads) vs swizzled rows (build/rev_swz);
# hardware-exp2 GRU gates (conv flag 256)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
SWZ="OFLOW_LIB=build/rev_swz/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/rev_swz/_lib/liboflow_torch.so"
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-events --no-step-flops"
tools/gpu_job.sh \
  "240|r4s15_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
  "120|r4s15_cb_pad|python -u tools/convbench.py" \
  "120|r4s15_cb_swz|$SWZ python -u tools/convbench.py" \
  "120|r4s15_cb_hw|python -u tools/convbench.py --conv-flags 256" \
  "120|r4s15_b_pad1|$B" "120|r4s15_b_swz1|$SWZ $B" "120|r4s15_b_pad2|$B" "120|r4s15_b_swz2|$SWZ $B" \
  "400|r4s15_ab|ATTRS='{\"lds\": {\"native:CONV_BREG\": false, \"lib:oflow_exp_set_conv_flags\": 0}, \"breg\": {\"native:CONV_BREG\": true, \"lib:oflow_exp_set_conv_flags\": 0}, \"breg_hw\": {\"native:CONV_BREG\": true, \"lib:oflow_exp_set_conv_flags\": 256}}' SAMPLES=8 python -u tools/exp/attr_ab.py"
