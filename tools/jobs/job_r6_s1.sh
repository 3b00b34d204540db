#!/usr/bin/env bash
# r06 s1: round-start state on a fresh box: GPU suite (new 1080p configs[4] test), smoke, default bench, hd bench
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "600|r6s1_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests -rA -k 'not zzz' 2>&1 | grep -v '^PASSED' " \
 "200|r6s1_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|r6s1_bench|python -u bench.py" \
 "200|r6s1_bench_hd|python -u bench.py --workload hd --no-cpu-baseline"
