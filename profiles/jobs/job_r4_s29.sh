#!/usr/bin/env bash
# r04 s29: stream structure re-check on the current kernels: pair lanes 2 / 3 / 4, fnet halves on one stream
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "600|r4s29_ab|ATTRS='{\"base\": {\"pair_lanes\": 2, \"fnet_streams\": true}, \"lanes3\": {\"pair_lanes\": 3, \"fnet_streams\": true}, \"lanes4\": {\"pair_lanes\": 4, \"fnet_streams\": true}, \"fnet1\": {\"pair_lanes\": 2, \"fnet_streams\": false}}' SAMPLES=6 python -u tools/exp/attr_ab.py"
