#!/usr/bin/env bash
# r03 s16: strip-walking warp: parity tests, timing vs the per-tile kernel
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|s16_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k warp" \
 "200|s16_warp_ab|HOOK=oflow_exp_set_warp_strip CPW=1,0 python -u tools/exp/run_warp_ab.py"
