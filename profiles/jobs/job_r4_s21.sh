#!/usr/bin/env bash
# r04 s21: XCD-aware workgroup order vs the 2D grid (build/rev_noxcd)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
NX="OFLOW_LIB=build/rev_noxcd/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/rev_noxcd/_lib/liboflow_torch.so"
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-events --no-step-flops"
tools/gpu_job.sh \
 "240|r4s21_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "120|r4s21_cb_x|python -u tools/convbench.py --no-lookup" \
 "120|r4s21_cb_nx|$NX python -u tools/convbench.py --no-lookup" \
 "120|r4s21_b_x1|$B" "120|r4s21_b_nx1|$NX $B" "120|r4s21_b_x2|$B" "120|r4s21_b_nx2|$NX $B"
