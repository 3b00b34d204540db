#!/usr/bin/env bash
# r05 s35: lane offset (OFLOW_LANE_OFFSET: lane 1 starts after lane 0 issued that stage of iteration 0), graph bench
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s35_none1|python -u bench.py --no-cpu-baseline" \
 "300|r5s35_mo1|OFLOW_LANE_OFFSET=mo python -u bench.py --no-cpu-baseline" \
 "300|r5s35_zr2a|OFLOW_LANE_OFFSET=zr2 python -u bench.py --no-cpu-baseline" \
 "300|r5s35_none2|python -u bench.py --no-cpu-baseline" \
 "300|r5s35_mo2|OFLOW_LANE_OFFSET=mo python -u bench.py --no-cpu-baseline" \
 "300|r5s35_zr2b|OFLOW_LANE_OFFSET=zr2 python -u bench.py --no-cpu-baseline"
