#!/usr/bin/env bash
# r04 s33: GraphedRAFT multi-pair capture with one lane (tests), and the 8-pair graph bench
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r4s33_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_raft.py -k 'graph'" \
 "200|r4s33_bench_graph8|python -u bench.py --no-cpu-baseline --graph"
