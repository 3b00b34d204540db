#!/usr/bin/env bash
# r06 s18: kernel trace of the eager 8-pair step (per-kernel breakdown and phases) on the current defaults
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r6s18_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6s18_prof -o run -- python3 bench.py --eager --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops" \
 "60|r6s18_phases|T=\$(find gpurun_out/r6s18_prof -name '*kernel_trace.csv' | head -1); python3 tools/step_phases.py \$T --steps 4 && python3 tools/prof_summary.py \$T --steps 6 --skip-last 2 > gpurun_out/r6s18_breakdown.txt; cp \$(find gpurun_out/r6s18_prof -name '*kernel_stats.csv' | head -1) gpurun_out/r6s18_kernel_stats.csv; rm -rf gpurun_out/r6s18_prof"
