#!/usr/bin/env bash
# r05 s47: encoder conv channel blocks re-checked on the graph bench (OFLOW_ENC_BN maps default blocks), alternated
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s47_base1|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s47_l3_64a|OFLOW_ENC_BN=128=64 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s47_l2_32a|OFLOW_ENC_BN=96=32 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s47_botha|OFLOW_ENC_BN=128=64,96=32 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s47_base2|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s47_l3_64b|OFLOW_ENC_BN=128=64 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s47_l2_32b|OFLOW_ENC_BN=96=32 python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s47_bothb|OFLOW_ENC_BN=128=64,96=32 python -u bench.py --no-cpu-baseline --no-step-flops"
