#!/usr/bin/env bash
# r05 s3: pipelined fused lookup + convc1 (variants 1 / 2 / 3 in-process A/B), GPU suite (two-lane graph capture,
# per-forward range snapshots), bench default + --graph
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r5s3_c1ab|VARIANTS=1,2,3 python -u tools/exp/run_c1_variant_ab.py" \
 "600|r5s3_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "300|r5s3_bench|python -u bench.py --no-cpu-baseline" \
 "300|r5s3_bench_graph|python -u bench.py --no-cpu-baseline --graph"
