#!/usr/bin/env bash
# r05 s41: split pyramid target-tile order A/B (blocked 4x2 vs row-major), full and epilogue alone, plus the fp32 pyramid
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh "300|r5s41_pyr_order|python -u tools/exp/pyr_order_probe.py"
