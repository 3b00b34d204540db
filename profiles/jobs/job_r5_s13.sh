#!/usr/bin/env bash
# r05 s13: quad-mapping variant 7 against 1 and 6
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r5s13_c1ab|VARIANTS=1,6,7 python -u tools/exp/run_c1_variant_ab.py" \
 "200|r5s13_stamps|VARIANTS=1,7 python -u tools/exp/run_c1_stamps_variants.py"
