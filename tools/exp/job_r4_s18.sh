#!/usr/bin/env bash
# r04 s18: where the BREG kernels' time goes (ablation build: MFMAs / A staging / epilogue dropped), and a fresh
# rocprof breakdown + phases of the step on the current build
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
ABL="OFLOW_LIB=build/rev_abl/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/rev_abl/_lib/liboflow_torch.so"
tools/gpu_job.sh \
 "200|r4s18_abl|$ABL python -u tools/convbench.py --ablate --no-lookup" \
 "300|r4s18_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4s18_prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops" \
 "60|r4s18_phases|T=\$(find gpurun_out/r4s18_prof -name '*kernel_trace.csv' | head -1); python3 tools/step_phases.py \$T --steps 4 && python3 tools/prof_summary.py \$T --steps 6 --skip-last 2 > gpurun_out/r4s18_breakdown.txt; rm -f \$T"
