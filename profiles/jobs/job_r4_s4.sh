#!/usr/bin/env bash
# r04 s4: pipelined steps (bench --inflight): test, bench 1 / 2 / 3 steps in flight, rocprof of inflight 2
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "300|r4s4_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_raft.py -k 'in_flight or range_guard or benchmarked or pair_lanes'" \
 "200|r4s4_bench_if1|python -u bench.py --no-cpu-baseline" \
 "200|r4s4_bench_if2|python -u bench.py --no-cpu-baseline --inflight 2" \
 "200|r4s4_bench_if3|python -u bench.py --no-cpu-baseline --inflight 3" \
 "200|r4s4_bench_if2b|python -u bench.py --no-cpu-baseline --inflight 2 --steps 20" \
 "200|r4s4_bench_if1b|python -u bench.py --no-cpu-baseline --steps 20" \
 "300|r4s4_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4s4_prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-step-flops --inflight 2" \
 "60|r4s4_sum|T=\$(find gpurun_out/r4s4_prof -name '*kernel_trace.csv' | head -1); python3 tools/prof_summary.py \$T --steps 6 --skip-last 2 > gpurun_out/r4s4_breakdown.txt; rm -f \$T"
