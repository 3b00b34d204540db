#!/usr/bin/env bash
# r05 s43: update-block conv channel blocks re-checked on the graph bench (OFLOW_CONV_BN overrides), alternated
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s43_base1|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s43_c2_96a|OFLOW_CONV_BN=c2=96 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s43_mo64a|OFLOW_CONV_BN=mo=64 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s43_fh1_64a|OFLOW_CONV_BN=fh1=64 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s43_base2|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s43_c2_96b|OFLOW_CONV_BN=c2=96 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s43_mo64b|OFLOW_CONV_BN=mo=64 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s43_fh1_64b|OFLOW_CONV_BN=fh1=64 python -u bench.py --no-cpu-baseline --no-step-flops"
