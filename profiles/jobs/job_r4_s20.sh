#!/usr/bin/env bash
# r04 s20: vertical-tap operand reuse (VSLIDE) in the register-direct 5x1 GRU convs vs re-reading (build/rev_novs)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
NV="OFLOW_LIB=build/rev_novs/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/rev_novs/_lib/liboflow_torch.so"
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-events --no-step-flops"
tools/gpu_job.sh \
 "240|r4s20_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "120|r4s20_cb_vs|python -u tools/convbench.py --no-lookup" \
 "120|r4s20_cb_nv|$NV python -u tools/convbench.py --no-lookup" \
 "120|r4s20_b_vs1|$B" "120|r4s20_b_nv1|$NV $B" "120|r4s20_b_vs2|$B" "120|r4s20_b_nv2|$NV $B"
