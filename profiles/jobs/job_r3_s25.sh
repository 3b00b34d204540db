#!/usr/bin/env bash
# r03 s25: 32-bit indexing in flow_prep / pack_s32: tests, step A/B vs HEAD
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
L() { echo "OFLOW_LIB=build/$1/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/$1/_lib/liboflow_torch.so"; }
tools/gpu_job.sh \
 "300|s25_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "120|s25_ab_new1|python -u tools/exp/step_ab.py" \
 "120|s25_ab_head1|$(L rev_head) python -u tools/exp/step_ab.py" \
 "120|s25_ab_new2|python -u tools/exp/step_ab.py" \
 "120|s25_ab_head2|$(L rev_head) python -u tools/exp/step_ab.py" \
 "300|s25_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s25_prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline" \
 "60|s25_phases|T=\$(find gpurun_out/s25_prof -name '*kernel_trace.csv' | head -1); python3 tools/step_phases.py \$T --steps 4 && python3 tools/prof_summary.py \$T --steps 6 --skip-last 2 > gpurun_out/s25_breakdown.txt; rm -rf gpurun_out/s25_prof"
