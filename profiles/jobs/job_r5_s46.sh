#!/usr/bin/env bash
# r05 s46: convc2 96 / fh1 64 channel blocks as the default: GPU suite, smoke, benches (KITTI against the old blocks)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tools/gpu_job.sh \
 "900|r5s46_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "200|r5s46_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|r5s46_bench|python -u bench.py" \
 "200|r5s46_bench2|python -u bench.py --no-cpu-baseline" \
 "200|r5s46_bench_eager|python -u bench.py --eager --no-cpu-baseline" \
 "300|r5s46_kitti_new|python -u bench.py --workload kitti --no-cpu-baseline --no-step-flops" \
 "300|r5s46_kitti_old|OFLOW_CONV_BN=c2=64,fh1=128 python -u bench.py --workload kitti --no-cpu-baseline --no-step-flops" \
 "200|r5s46_bench_hd|python -u bench.py --workload hd --no-cpu-baseline"
