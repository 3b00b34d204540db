#!/usr/bin/env bash
# r06 s25: the final tree (early lane state): smoke, the default bench (with cpu_baseline), a second default bench,
# KITTI and hd
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "200|r6s25_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|r6s25_bench|python -u bench.py" \
 "200|r6s25_bench2|python -u bench.py --no-cpu-baseline" \
 "300|r6s25_bench_kitti|python -u bench.py --workload kitti --no-cpu-baseline" \
 "200|r6s25_bench_hd|python -u bench.py --workload hd --no-cpu-baseline"
