#!/usr/bin/env bash
# r05 s24: pair lanes under graph replay: 1 / 2 / 4 lanes, interleaved
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s24_l2a|python -u bench.py --no-cpu-baseline --lanes 2" \
 "300|r5s24_l1a|python -u bench.py --no-cpu-baseline --lanes 1" \
 "300|r5s24_l4a|python -u bench.py --no-cpu-baseline --lanes 4" \
 "300|r5s24_l2b|python -u bench.py --no-cpu-baseline --lanes 2" \
 "300|r5s24_l1b|python -u bench.py --no-cpu-baseline --lanes 1" \
 "300|r5s24_l4b|python -u bench.py --no-cpu-baseline --lanes 4"
