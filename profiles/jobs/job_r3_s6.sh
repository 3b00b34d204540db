#!/usr/bin/env bash
# r03 session 6: HEAD GPU suite, the vectorizer build-flag A/B (lane determinism + step time), bench
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
V=build/vec/_lib
tools/gpu_job.sh \
 "700|r3_s6_pytest|python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests" \
 "300|r3_s6_vec_lanes|OFLOW_LIB=$V/liboflow_hip.so OFLOW_OPS_LIB=$V/liboflow_torch.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_corr_convc1.py tests/test_gpu_raft.py tests/test_gpu_parity.py" \
 "120|r3_s6_ab_base1|python -u tools/exp/step_ab.py" \
 "120|r3_s6_ab_vec1|OFLOW_LIB=$V/liboflow_hip.so OFLOW_OPS_LIB=$V/liboflow_torch.so python -u tools/exp/step_ab.py" \
 "120|r3_s6_ab_base2|python -u tools/exp/step_ab.py" \
 "120|r3_s6_ab_vec2|OFLOW_LIB=$V/liboflow_hip.so OFLOW_OPS_LIB=$V/liboflow_torch.so python -u tools/exp/step_ab.py" \
 "300|r3_s6_bench|python -u bench.py"
