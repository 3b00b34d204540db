#!/usr/bin/env bash
# r04 s18: 3-deep B ring for the register-direct kernels vs 2 (build/rev_r2); where their time goes (ablation build,
# ring 2); a fresh rocprof breakdown + phases of the step on the current build
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
ABL="OFLOW_LIB=build/rev_abl/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/rev_abl/_lib/liboflow_torch.so"
R2="OFLOW_LIB=build/rev_r2/_lib/liboflow_hip.so OFLOW_OPS_LIB=build/rev_r2/_lib/liboflow_torch.so"
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-events --no-step-flops"
tools/gpu_job.sh \
 "240|r4s18_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "120|r4s18_cb_r3|python -u tools/convbench.py --no-lookup" \
 "120|r4s18_cb_r2|$R2 python -u tools/convbench.py --no-lookup" \
 "120|r4s18_b_r3a|$B" "120|r4s18_b_r2a|$R2 $B" "120|r4s18_b_r3b|$B" "120|r4s18_b_r2b|$R2 $B" \
 "200|r4s18_abl|$ABL python -u tools/convbench.py --ablate --no-lookup" \
 "300|r4s18_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4s18_prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops" \
 "60|r4s18_phases|T=\$(find gpurun_out/r4s18_prof -name '*kernel_trace.csv' | head -1); python3 tools/step_phases.py \$T --steps 4 && python3 tools/prof_summary.py \$T --steps 6 --skip-last 2 > gpurun_out/r4s18_breakdown.txt; rm -f \$T"
