#!/usr/bin/env bash
# r04 s12: where the 8-pair graph capture crashes (Python stack via faulthandler)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r4s12_graph8|python -X faulthandler -u bench.py --no-cpu-baseline --graph --steps 2 --warmup 1"
