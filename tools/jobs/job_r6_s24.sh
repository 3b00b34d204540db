#!/usr/bin/env bash
# r06 s24: the pair lanes' SplitUpdate state built on the cnet stream beside the pyramid (raft.EARLY_LANE_INIT):
# GPU suite, in-process graph A/B alternated (off / on), eager bench with the new default
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "600|r6s24_pytest|python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "400|r6s24_ab|VARIANTS='off:raft.EARLY_LANE_INIT=False;on:raft.EARLY_LANE_INIT=True' ROUNDS=8 python3 -u tools/exp/run_graph_ab.py" \
 "200|r6s24_eager|python3 -u bench.py --eager --steps 40 --warmup 5 --no-cpu-baseline --no-step-flops"
