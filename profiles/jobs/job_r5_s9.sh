#!/usr/bin/env bash
# r05 s9: timing events recorded inside a captured HIP graph (external events) -- usable for bench.py --graph's roofline?
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh "200|r5s9_graph_events|python -X faulthandler -u tools/exp/graph_event_probe.py"
