#!/usr/bin/env bash
# r04 s40: cnet beside the pyramid (after fnet) vs beside fnet
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "120|r4s40_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_raft.py -k 'golden or batch or lanes'" \
 "500|r4s40_ab|ATTRS='{\"beside_fnet\": {\"cnet_after_fnet\": false}, \"beside_pyramid\": {\"cnet_after_fnet\": true}}' SAMPLES=10 python -u tools/exp/attr_ab.py"
