#!/usr/bin/env bash
# r05 s45: the leading conv channel-block sets, alternated three times on the graph bench (OFLOW_CONV_BN overrides)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
A="c2=96"; C="c2=96,mo=64,fh1=64"; E="c2=96,fh1=64"
tools/gpu_job.sh \
 "300|r5s45_a1|OFLOW_CONV_BN=$A python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s45_c1|OFLOW_CONV_BN=$C python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s45_e1|OFLOW_CONV_BN=$E python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s45_a2|OFLOW_CONV_BN=$A python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s45_c2|OFLOW_CONV_BN=$C python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s45_e2|OFLOW_CONV_BN=$E python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s45_a3|OFLOW_CONV_BN=$A python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s45_c3|OFLOW_CONV_BN=$C python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s45_e3|OFLOW_CONV_BN=$E python -u bench.py --no-cpu-baseline --no-step-flops"
