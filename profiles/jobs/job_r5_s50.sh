#!/usr/bin/env bash
# r05 s50: conv channel blocks chosen by where the flow branch runs (side stream: the r04 blocks; inline, as in the
# replayed graph: convc2 96 / fh1 64): eager and graph benches, RAFT GPU tests
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "600|r5s50_test|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_raft.py" \
 "300|r5s50_graph1|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s50_eager1|python -u bench.py --eager --no-cpu-baseline --no-step-flops" \
 "300|r5s50_graph2|python -u bench.py --no-cpu-baseline --no-step-flops" \
 "300|r5s50_eager2|python -u bench.py --eager --no-cpu-baseline --no-step-flops"
