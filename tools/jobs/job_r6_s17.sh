#!/usr/bin/env bash
# r06 s17: the new defaults (LDS-staged convs with 2-step operand prefetch, unconditional-load warp and lookup):
# whole GPU suite, smoke, default bench
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "900|r6s17_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests -rf" \
 "200|r6s17_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|r6s17_bench|python -u bench.py"
