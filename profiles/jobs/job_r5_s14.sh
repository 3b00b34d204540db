#!/usr/bin/env bash
# r05 s14: 128-query variant 8 against 1 and 7
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r5s14_c1ab|VARIANTS=1,7,8 python -u tools/exp/run_c1_variant_ab.py" \
 "200|r5s14_stamps|VARIANTS=1,8 python -u tools/exp/run_c1_stamps_variants.py"
