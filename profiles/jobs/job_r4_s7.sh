#!/usr/bin/env bash
# r04 s7: hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4) for the forward's 6 streams
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r4s7_q4|GPU_MAX_HW_QUEUES=4 python -u bench.py --no-cpu-baseline" \
 "200|r4s7_q8|GPU_MAX_HW_QUEUES=8 python -u bench.py --no-cpu-baseline" \
 "200|r4s7_q16|GPU_MAX_HW_QUEUES=16 python -u bench.py --no-cpu-baseline" \
 "200|r4s7_q4b|GPU_MAX_HW_QUEUES=4 python -u bench.py --no-cpu-baseline" \
 "200|r4s7_q8b|GPU_MAX_HW_QUEUES=8 python -u bench.py --no-cpu-baseline" \
 "200|r4s7_q8_if2|GPU_MAX_HW_QUEUES=8 python -u bench.py --no-cpu-baseline --inflight 2"
