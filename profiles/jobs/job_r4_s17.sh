#!/usr/bin/env bash
# PMC (MFMA / VALU / LDS / waits) of the step's MFMA kernels on the current build, then a bench
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "400|r4s17_pmcm|bash tools/pmc_mfma_job.sh" \
 "60|r4s17_pmcm_sum|python3 tools/pmc_mfma.py \$(find gpurun_out/pmcm/p1 -name '*counter_collection.csv' | head -1) \$(find gpurun_out/pmcm/p2 -name '*counter_collection.csv' | head -1) --json gpurun_out/r4s17_pmc_mfma.json; find gpurun_out/pmcm -name '*.csv' -size +20M -delete" \
 "120|r4s17_b1|python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-events --no-step-flops"
