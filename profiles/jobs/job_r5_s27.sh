#!/usr/bin/env bash
# r05 s27: graph capture with a live RCCL communicator (world 1 over nccl)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh "300|r5s27_probe|python -u tools/exp/graph_rccl_probe.py"
