#!/usr/bin/env bash
# r04 s11: GraphedRAFT (capture on the warm-up stream): batch-1 tests, then the 8-pair bench from a HIP graph
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r4s11_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_raft.py -k 'graphed or range_guard_deferred'" \
 "200|r4s11_b1graph|python -u bench.py --no-cpu-baseline --pairs-per-gpu 1 --iters 24 --graph" \
 "200|r4s11_graph8|python -u bench.py --no-cpu-baseline --graph"
