#!/usr/bin/env bash
# r05 s11: checkpoint after moving the convc1 variants out of the product: GPU suite, smoke, bench, variant A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "600|r5s11_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "200|r5s11_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|r5s11_bench|python -u bench.py" \
 "200|r5s11_c1ab|VARIANTS=1,2,5 python -u tools/exp/run_c1_variant_ab.py"
