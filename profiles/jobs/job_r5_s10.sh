#!/usr/bin/env bash
# r05 s10: 2-row tiles for the q convs (flag 512) and the motion conv (flag 1024): step A/B in-process, convbench of both
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "400|r5s10_ab|FLAGS=0,512,1024,1536 python -u tools/exp/run_conv_flags_ab.py" \
 "200|r5s10_cb|python -u tools/convbench.py"
