#!/usr/bin/env bash
# r06 s14: warp strip kernel with unconditional (buffer, sentinel) row loads vs the r03 form, bit-identity, A/B
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "180|r6s14_warp_ab|HOOK=oflow_exp_set_warp_strip CPW=1,2 python -u tools/exp/run_warp_ab.py"
