#!/usr/bin/env bash
# r04 s39: pack_s32 with one thread per pixel x 32 channels: tests, two benches
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r4s39_tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s32.py tests/test_gpu_raft.py" \
 "200|r4s39_bench|python -u bench.py --no-cpu-baseline" \
 "200|r4s39_bench2|python -u bench.py --no-cpu-baseline"
