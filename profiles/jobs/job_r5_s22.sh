#!/usr/bin/env bash
# r05 s22: rocprof kernel trace of bench --graph (do the in-graph event timings agree with the trace?) + its phases
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s22_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5s22_prof -o run -- python3 bench.py --graph --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops" \
 "60|r5s22_phases|T=\$(find gpurun_out/r5s22_prof -name '*kernel_trace.csv' | head -1); python3 tools/step_phases.py \$T --steps 4 && python3 tools/prof_summary.py \$T --steps 6 --skip-last 2 > gpurun_out/r5s22_breakdown.txt; cp \$(find gpurun_out/r5s22_prof -name '*kernel_stats.csv' | head -1) gpurun_out/r5s22_kernel_stats.csv; python3 tools/exp/lane_overlap.py \$T > gpurun_out/r5s22_overlap.txt; rm -f \$T"
