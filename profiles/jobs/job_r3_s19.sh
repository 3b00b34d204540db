#!/usr/bin/env bash
# r03 s19: cnet started part-way through fnet (its tail overlapping the corr pyramid)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "400|s19_ab_cnet_delay|SAMPLES=6 ATTRS='{\"d0\": {\"cnet_delay\": 0}, \"d1\": {\"cnet_delay\": 1}, \"d2\": {\"cnet_delay\": 2}, \"d3\": {\"cnet_delay\": 3}, \"d4\": {\"cnet_delay\": 4}, \"d0_\": {\"cnet_delay\": 0}}' python -u tools/exp/attr_ab.py"
