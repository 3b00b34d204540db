#!/usr/bin/env bash
# r04 s10: the bench's own per-launch HIP events (fused lookup + pyramid) vs none, at 4 and 8 hardware queues
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r4s10_ev_q4|python -u bench.py --no-cpu-baseline" \
 "200|r4s10_noev_q4|python -u bench.py --no-cpu-baseline --no-events" \
 "200|r4s10_ev_q8|GPU_MAX_HW_QUEUES=8 python -u bench.py --no-cpu-baseline" \
 "200|r4s10_noev_q8|GPU_MAX_HW_QUEUES=8 python -u bench.py --no-cpu-baseline --no-events" \
 "200|r4s10_ev_q4b|python -u bench.py --no-cpu-baseline" \
 "200|r4s10_noev_q4b|python -u bench.py --no-cpu-baseline --no-events"
