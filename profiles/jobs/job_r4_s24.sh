#!/usr/bin/env bash
# r04 s24: the stem with one A buffer (three workgroups per CU) vs two (build/rev_stem2): encoders alone and the step
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
S2="OFLOW_LIB=build/rev_stem2/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/rev_stem2/_lib/liboflow_torch.so"
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-events --no-step-flops"
tools/gpu_job.sh \
 "300|r4s24_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_raft.py tests/test_gpu_conv_s32.py" \
 "120|r4s24_enc1|python -u tools/exp/enc_bench.py" "120|r4s24_enc2|$S2 python -u tools/exp/enc_bench.py" \
 "120|r4s24_enc1b|python -u tools/exp/enc_bench.py" "120|r4s24_enc2b|$S2 python -u tools/exp/enc_bench.py" \
 "120|r4s24_b1|$B" "120|r4s24_b2|$S2 $B" "120|r4s24_b1b|$B" "120|r4s24_b2b|$S2 $B"
