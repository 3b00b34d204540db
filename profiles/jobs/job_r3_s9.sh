#!/usr/bin/env bash
# r03 s9: BN64 8-row tiles in-step A/B; rocprof kernel trace of the bench step (phases, breakdown)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|s9_ab_bn64|SAMPLES=8 ATTRS='{\"r8\": {}, \"r4\": {\"lib:oflow_exp_set_bn64_8row\": 0}, \"r8_\": {\"lib:oflow_exp_set_bn64_8row\": 1}}' python -u tools/exp/attr_ab.py" \
 "300|s9_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s9_prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline" \
 "60|s9_phases|T=\$(find gpurun_out/s9_prof -name '*kernel_trace.csv' | head -1); python3 tools/step_phases.py \$T --steps 3 && python3 tools/prof_summary.py \$T --steps 4 --skip-last 2 > gpurun_out/s9_breakdown.txt"
