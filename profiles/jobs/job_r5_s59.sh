#!/usr/bin/env bash
# r05 s59: 8-row tiles for the instance-norm convs on by default: GPU suite, smoke, graph and eager benches against
# oflow_exp_set_stats_8row(0) (the 4-row tiles), alternated
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OLD="OFLOW_EXP_CALLS='oflow_exp_set_stats_8row=0'"
tools/gpu_job.sh \
 "900|r5s59_pytest|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests" \
 "200|r5s59_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|r5s59_new1|python -u bench.py" \
 "300|r5s59_old1|$OLD python -u bench.py --no-cpu-baseline" \
 "300|r5s59_new2|python -u bench.py --no-cpu-baseline" \
 "300|r5s59_old2|$OLD python -u bench.py --no-cpu-baseline" \
 "300|r5s59_eager_new|python -u bench.py --eager --no-cpu-baseline --no-step-flops" \
 "300|r5s59_eager_old|$OLD python -u bench.py --eager --no-cpu-baseline --no-step-flops" \
 "300|r5s59_kitti|python -u bench.py --workload kitti --no-cpu-baseline"
