#!/usr/bin/env bash
# r05 s15: product fused kernel = the quad mapping (variant 7): GPU suite, A/B against variants 5/7 (bit identity), bench
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "600|r5s15_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "200|r5s15_c1ab|VARIANTS=1,5,7 python -u tools/exp/run_c1_variant_ab.py" \
 "300|r5s15_bench|python -u bench.py" \
 "300|r5s15_bench2|python -u bench.py --no-cpu-baseline"
