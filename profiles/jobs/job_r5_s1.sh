#!/usr/bin/env bash
# r05 s1: two-lane graph capture probe (flag fix; then lane buffers on main) + the graph tests
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "240|r5s1_probe_flag|VARIANT=flag PAIRS=8 python -X faulthandler -u tools/exp/graph_lanes_probe.py" \
 "240|r5s1_probe_initmain|VARIANT=initmain PAIRS=8 python -X faulthandler -u tools/exp/graph_lanes_probe.py" \
 "300|r5s1_graph_tests|python -X faulthandler -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_raft.py -k graphed"
