#!/usr/bin/env bash
# r05 s38: store-bandwidth reference for the split pyramid epilogue (fill / copy / pyramid / epilogue alone)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh "300|r5s38_store_bw|python -u tools/exp/store_bw_probe.py"
