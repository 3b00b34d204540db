#!/usr/bin/env bash
# r05 s39: split pyramid epilogue ablations (level 0 alone, unstaged stores) vs a fill
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh "300|r5s39_pyr_epi|python -u tools/exp/pyr_epi_probe.py"
