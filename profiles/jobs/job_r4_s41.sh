#!/usr/bin/env bash
# r04 s41: the committed final tree: full GPU suite and smoke
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "900|r4s41_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "200|r4s41_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|r4s41_bench|python -u bench.py"
