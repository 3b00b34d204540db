#!/usr/bin/env bash
# r05 s55: configs[4] (1 pair 1080x1920, on-the-fly fp16 correlation) replayed from a HIP graph vs eager, alternated
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s55_eager1|python -u bench.py --workload hd --no-cpu-baseline --no-step-flops" \
 "300|r5s55_graph1|python -u bench.py --workload hd --graph --no-cpu-baseline --no-step-flops" \
 "300|r5s55_eager2|python -u bench.py --workload hd --no-cpu-baseline --no-step-flops" \
 "300|r5s55_graph2|python -u bench.py --workload hd --graph --no-cpu-baseline --no-step-flops"
