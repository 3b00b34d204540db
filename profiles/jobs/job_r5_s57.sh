#!/usr/bin/env bash
# r05 s57: register-direct weights for the 64-channel 3x3 blocks (OFLOW_CONV_BREG64=1: convf2, the flow head's first
# conv) on the graph bench, alternated against the default (LDS-staged B for those blocks)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s57_base1|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s57_breg1|OFLOW_CONV_BREG64=1 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s57_base2|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s57_breg2|OFLOW_CONV_BREG64=1 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s57_base3|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s57_breg3|OFLOW_CONV_BREG64=1 python -u bench.py --no-cpu-baseline --no-step-flops"
