#!/usr/bin/env bash
# r05 s58: 8-row tiles for the 64-channel convs (oflow_exp_set_bn64_8row: convf2, the flow head's first conv, cnet's
# layer 1; oflow_exp_set_stats_8row: fnet's instance-norm layer-1 convs) re-checked on the graph bench, alternated
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s58_base1|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s58_bn64a|OFLOW_EXP_CALLS='oflow_exp_set_bn64_8row=1' python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s58_statsa|OFLOW_EXP_CALLS='oflow_exp_set_stats_8row=1' python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s58_base2|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s58_bn64b|OFLOW_EXP_CALLS='oflow_exp_set_bn64_8row=1' python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s58_statsb|OFLOW_EXP_CALLS='oflow_exp_set_stats_8row=1' python -u bench.py --no-cpu-baseline --no-step-flops"
