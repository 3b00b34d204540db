#!/usr/bin/env bash
# r04 s38: the committed final tree (native InputPadder pad included): GPU suite, smoke, two benches
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "900|r4s38_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "200|r4s38_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|r4s38_bench|python -u bench.py" \
 "200|r4s38_bench2|python -u bench.py --no-cpu-baseline"
