#!/usr/bin/env bash
# r05 s44: update-block conv channel blocks, combinations on the graph bench (OFLOW_CONV_BN overrides), alternated
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
A="c2=96"; B="c2=96,mo=64"; C="c2=96,mo=64,fh1=64"; D="c2=96,mo=64,f2=32"
tools/gpu_job.sh \
 "300|r5s44_a1|OFLOW_CONV_BN=$A python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s44_b1|OFLOW_CONV_BN=$B python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s44_c1|OFLOW_CONV_BN=$C python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s44_d1|OFLOW_CONV_BN=$D python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s44_a2|OFLOW_CONV_BN=$A python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s44_b2|OFLOW_CONV_BN=$B python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s44_c2|OFLOW_CONV_BN=$C python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s44_d2|OFLOW_CONV_BN=$D python -u bench.py --no-cpu-baseline --no-step-flops"
