#!/usr/bin/env bash
# r05 s7: hybrid fused lookup + convc1 (variant 5) vs the r04 kernel: A/B (bit identity), stamps
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r5s7_c1ab|VARIANTS=1,5 python -u tools/exp/run_c1_variant_ab.py" \
 "200|r5s7_stamps|VARIANTS=1,5 python -u tools/exp/run_c1_stamps_variants.py"
