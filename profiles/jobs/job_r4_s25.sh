#!/usr/bin/env bash
# r04 s25: pyramid epilogue with 32-bit offsets vs before (build/rev_pyrbase = HEAD~2): kernel alone and the step;
# encoder 8-row tile variants (stats / plain BN-64 convs) in-process
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
PB="OFLOW_LIB=build/rev_pyrbase/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/rev_pyrbase/_lib/liboflow_torch.so"
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-events --no-step-flops"
tools/gpu_job.sh \
 "300|r4s25_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pyramid_s32.py tests/test_gpu_parity.py tests/test_gpu_raft.py" \
 "120|r4s25_kb|python -u tools/kbench.py" "120|r4s25_kb0|$PB python -u tools/kbench.py" \
 "120|r4s25_kbb|python -u tools/kbench.py" "120|r4s25_kb0b|$PB python -u tools/kbench.py" \
 "120|r4s25_b1|$B" "120|r4s25_b0|$PB $B" "120|r4s25_b1b|$B" "120|r4s25_b0b|$PB $B" \
 "300|r4s25_enc|ARMS='{\"base\": {}, \"s8\": {\"oflow_exp_set_stats_8row\": 1}, \"b8\": {\"oflow_exp_set_bn64_8row\": 1}, \"s8b8\": {\"oflow_exp_set_stats_8row\": 1, \"oflow_exp_set_bn64_8row\": 1}}' python -u tools/exp/enc_bench.py"
