#!/usr/bin/env bash
# r06 s29: the after-step legs (API lookup, warp) timed as back-to-back launches between one event pair: the default
# bench, and the eager bench under rocprofv3 (the legs' event times against rocprof's kernel means, same command)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r6s29_bench|python -u bench.py --no-cpu-baseline" \
 "300|r6s29_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6s29_prof -o run -- python3 bench.py --eager --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops" \
 "60|r6s29_stats|cp \$(find gpurun_out/r6s29_prof -name '*kernel_stats.csv' | head -1) gpurun_out/r6s29_kernel_stats.csv; rm -rf gpurun_out/r6s29_prof"
