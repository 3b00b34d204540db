#!/usr/bin/env bash
# r05 s8: rocprof kernel trace + phases of the default bench (current tree), for the step breakdown
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s8_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5s8_prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops" \
 "60|r5s8_phases|T=\$(find gpurun_out/r5s8_prof -name '*kernel_trace.csv' | head -1); python3 tools/step_phases.py \$T --steps 4 && python3 tools/prof_summary.py \$T --steps 6 --skip-last 2 > gpurun_out/r5s8_breakdown.txt; cp \$(find gpurun_out/r5s8_prof -name '*kernel_stats.csv' | head -1) gpurun_out/r5s8_kernel_stats.csv; rm -f \$T"
