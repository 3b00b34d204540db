#!/usr/bin/env bash
# r04 s32: GraphedRAFT at 8 pairs with one pair lane (the two-lane capture crashed in capture_end at s5/s6)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh "300|r4s32_graph8l1|PAIRS=8 LANES=1 python -u tools/exp/graph_probe.py"
