#!/usr/bin/env bash
# r05 s51: eager forward (flow branch on side streams) with the r04 blocks (CONV_BN_SIDE, the default there) vs convc2 96
# / fh1 64, alternated
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s51_old1|python -u bench.py --eager --no-cpu-baseline --no-step-flops" \
 "300|r5s51_new1|OFLOW_CONV_BN=c2=96,fh1=64 python -u bench.py --eager --no-cpu-baseline --no-step-flops" \
 "300|r5s51_old2|python -u bench.py --eager --no-cpu-baseline --no-step-flops" \
 "300|r5s51_new2|OFLOW_CONV_BN=c2=96,fh1=64 python -u bench.py --eager --no-cpu-baseline --no-step-flops" \
 "300|r5s51_old3|python -u bench.py --eager --no-cpu-baseline --no-step-flops" \
 "300|r5s51_new3|OFLOW_CONV_BN=c2=96,fh1=64 python -u bench.py --eager --no-cpu-baseline --no-step-flops"
