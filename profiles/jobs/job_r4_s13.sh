#!/usr/bin/env bash
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh "300|r4s13_phase|python -u tools/exp/phase_probe.py"
