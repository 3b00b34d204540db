#!/usr/bin/env bash
# r05 s53: three pair lanes (3 / 3 / 2 pairs) under graph replay against the default two, alternated
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s53_l2a|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s53_l3a|python -u bench.py --no-cpu-baseline --no-step-flops --lanes 3" \
 "300|r5s53_l2b|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s53_l3b|python -u bench.py --no-cpu-baseline --no-step-flops --lanes 3"
