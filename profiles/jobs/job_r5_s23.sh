#!/usr/bin/env bash
# r05 s23: graph replay as the bench default: default bench x2, --eager, kitti (graph), smoke
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s23_bench|python -u bench.py" \
 "300|r5s23_eager|python -u bench.py --eager --no-cpu-baseline" \
 "300|r5s23_bench2|python -u bench.py --no-cpu-baseline" \
 "300|r5s23_kitti|python -u bench.py --workload kitti --no-cpu-baseline" \
 "300|r5s23_conv|python -u bench.py --conv-events --no-cpu-baseline --steps 5"
