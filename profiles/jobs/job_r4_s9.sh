#!/usr/bin/env bash
# r04 s9: stream structure A/B (flow-branch side streams, pair lanes, encoder streams) at 4 and 8 hardware queues
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
A='{"base": {}, "noside": {"update_block.split_streams": false}, "lanes1": {"pair_lanes": 1}, "noside_lanes1": {"update_block.split_streams": false, "pair_lanes": 1}, "noenc": {"encoder_streams": false}, "nofnet2": {"fnet_streams": false}}'
tools/gpu_job.sh \
 "400|r4s9_ab_q4|GPU_MAX_HW_QUEUES=4 ATTRS='$A' SAMPLES=5 python -u tools/exp/attr_ab.py" \
 "400|r4s9_ab_q8|GPU_MAX_HW_QUEUES=8 ATTRS='$A' SAMPLES=5 python -u tools/exp/attr_ab.py"
