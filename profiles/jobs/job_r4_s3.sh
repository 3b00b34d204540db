#!/usr/bin/env bash
# r04 s3: fused lookup + convc1 with lane-per-query gathers (old vs new in-process A/B, bit-identical), tests, bench
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r4s3_c1ab|OLD_LIB=build/rev_base/_lib/liboflow_hip.so python -u tools/exp/run_c1_rev_ab.py" \
 "600|r4s3_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_corr_convc1.py tests/test_gpu_raft.py" \
 "300|r4s3_bench|python -u bench.py --no-cpu-baseline" \
 "300|r4s3_bench2|python -u bench.py --no-cpu-baseline"
