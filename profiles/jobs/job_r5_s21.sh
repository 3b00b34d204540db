#!/usr/bin/env bash
# r05 s21: bench --graph with per-kernel native event nodes in the graph (roofline in graph mode) vs eager, same box
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s21_graph|python -u bench.py --graph --no-cpu-baseline" \
 "300|r5s21_eager|python -u bench.py --no-cpu-baseline" \
 "300|r5s21_graph2|python -u bench.py --graph --no-cpu-baseline" \
 "300|r5s21_eager2|python -u bench.py --no-cpu-baseline"
