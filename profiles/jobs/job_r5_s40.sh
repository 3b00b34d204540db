#!/usr/bin/env bash
# r05 s40: split pyramid epilogue ablations (no level-3 / level 1-3 stores)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh "300|r5s40_pyr_epi|python -u tools/exp/pyr_epi_probe.py"
