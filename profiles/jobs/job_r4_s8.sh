#!/usr/bin/env bash
# r04 s8: fewer hardware queues per process (GPU_MAX_HW_QUEUES 1 / 2 / 3 vs the default 4)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r4s8_q4|GPU_MAX_HW_QUEUES=4 python -u bench.py --no-cpu-baseline" \
 "200|r4s8_q3|GPU_MAX_HW_QUEUES=3 python -u bench.py --no-cpu-baseline" \
 "200|r4s8_q2|GPU_MAX_HW_QUEUES=2 python -u bench.py --no-cpu-baseline" \
 "200|r4s8_q1|GPU_MAX_HW_QUEUES=1 python -u bench.py --no-cpu-baseline" \
 "200|r4s8_q5|GPU_MAX_HW_QUEUES=5 python -u bench.py --no-cpu-baseline" \
 "200|r4s8_q6|GPU_MAX_HW_QUEUES=6 python -u bench.py --no-cpu-baseline"
