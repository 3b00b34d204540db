#!/usr/bin/env bash
# r04 s36: ATen-on-GPU scalar division vs the true quotient (the native input scaling differs from ATen-GPU in s35)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh "120|r4s36_div|python -u tools/exp/div_check.py"
