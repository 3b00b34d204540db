#!/usr/bin/env bash
# r06 s15: warp strip kernel BUF variant (unconditional loads, flow 3 steps ahead, deferred out-of-ring pixels) vs r03;
# tiled lookup with unconditional buffer-load gathers vs r02
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "180|r6s15_warp_ab|HOOK=oflow_exp_set_warp_strip CPW=1,2 python -u tools/exp/run_warp_ab.py" \
 "180|r6s15_lookup_ab|python -u tools/exp/run_lookup_buf_ab.py"
