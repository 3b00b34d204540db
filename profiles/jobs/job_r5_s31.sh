#!/usr/bin/env bash
# r05 s31: convf1 straight from coords1 (OFLOW_IN_FLOW7) vs the patch-matrix path (OFLOW_CONVF1_FROM_FLOW=0), same
# library, interleaved whole-step A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r5s31_new1|python -u tools/exp/step_ab.py" \
 "200|r5s31_old1|OFLOW_CONVF1_FROM_FLOW=0 python -u tools/exp/step_ab.py" \
 "200|r5s31_new2|python -u tools/exp/step_ab.py" \
 "200|r5s31_old2|OFLOW_CONVF1_FROM_FLOW=0 python -u tools/exp/step_ab.py" \
 "200|r5s31_new3|python -u tools/exp/step_ab.py" \
 "200|r5s31_old3|OFLOW_CONVF1_FROM_FLOW=0 python -u tools/exp/step_ab.py" \
 "300|r5s31_bench|python -u bench.py --no-cpu-baseline"
