#!/usr/bin/env bash
# r04 s2: flow head as 1x1 conv + col2im, stem window de-interleaved in LDS: tests, in-process A/B, bench, rocprof
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "600|r4s2_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py tests/test_gpu_corr_convc1.py" \
 "300|r4s2_ab_fh|ATTRS='{\"col2im\": {\"mod:model.update.FLOW_HEAD_MODE\": \"col2im\"}, \"conv\": {\"mod:model.update.FLOW_HEAD_MODE\": \"conv\"}}' SAMPLES=8 python -u tools/exp/attr_ab.py" \
 "300|r4s2_bench|python -u bench.py --no-cpu-baseline" \
 "300|r4s2_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4s2_prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops" \
 "60|r4s2_phases|T=\$(find gpurun_out/r4s2_prof -name '*kernel_trace.csv' | head -1); python3 tools/step_phases.py \$T --steps 4 && python3 tools/prof_summary.py \$T --steps 6 --skip-last 2 > gpurun_out/r4s2_breakdown.txt; rm -f \$T"
