#!/usr/bin/env bash
# r03 s23: pair lanes started offset (lane 1 waits for part of lane 0's first iteration)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "400|s23_ab_lane_offset|SAMPLES=6 ATTRS='{\"o0\": {\"lane_offset\": 0}, \"o1\": {\"lane_offset\": 1}, \"o2\": {\"lane_offset\": 2}, \"o3\": {\"lane_offset\": 3}, \"o0_\": {\"lane_offset\": 0}}' python -u tools/exp/attr_ab.py"
