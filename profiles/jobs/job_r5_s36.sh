#!/usr/bin/env bash
# r05 s36: two graph captures in flight (bench.py --graph --inflight 2: step i replays capture i % 2 on stream i % 2),
# with 2 pair lanes and with 1, against the default (one capture, inflight 1)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r5s36_base1|python -u bench.py --no-cpu-baseline" \
 "300|r5s36_if2a|python -u bench.py --no-cpu-baseline --graph --inflight 2" \
 "300|r5s36_if2l1a|python -u bench.py --no-cpu-baseline --graph --inflight 2 --lanes 1" \
 "300|r5s36_base2|python -u bench.py --no-cpu-baseline" \
 "300|r5s36_if2b|python -u bench.py --no-cpu-baseline --graph --inflight 2" \
 "300|r5s36_if2l1b|python -u bench.py --no-cpu-baseline --graph --inflight 2 --lanes 1"
