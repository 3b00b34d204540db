#!/usr/bin/env bash
# r05 s19: split pyramid start-stagger A/B (tools/exp/run_pyr_stagger_ab.py)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh "300|r5s19b_stagger|EPI_ONLY=1 python -u tools/exp/run_pyr_stagger_ab.py"
