#!/usr/bin/env bash
# r05 s20: native timing events recorded inside a captured graph (external event nodes)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh "200|r5s20_probe|python -u tools/exp/graph_native_event_probe.py"
