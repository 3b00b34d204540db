#!/usr/bin/env bash
# r04 s6: host enqueue time vs GPU time; bench eager vs HIP graph at 8 pairs
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r4s6_host|python -u tools/exp/host_time.py" \
 "300|r4s6_bench_graph|python -u bench.py --no-cpu-baseline --graph" \
 "300|r4s6_bench_eager|python -u bench.py --no-cpu-baseline"
